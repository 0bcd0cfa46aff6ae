"""Isolated timing of the small weight gradients of the B=32 step (head
to_feature_map and the three skip projections, bias included):
dW[N, K] = dy^T x, db = colsum(dy) over tall M.  Env knobs of the library
(HVIT_NO_RS, HVIT_RING, ...) select the variant for A/B runs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib
HF = sys.modules["hvit_amd.functional"]
SHAPES = [("head", 2048, 256, 512), ("skip0", 8192, 256, 256), ("skip1", 32768, 128, 128),
          ("skip2", 131072, 64, 64)]
reps = 30
for name, M, N, K in SHAPES:
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    dw, db = HF.linear_wgrad(L.BF16, dy, x, M, N, K, bias=True)
    ref = dy.float().t() @ x.float()
    err = ((dw - ref).abs().max() / ref.abs().max()).item()
    errb = ((db - dy.float().sum(0)).abs().max() / dy.float().sum(0).abs().max()).item()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):  # back-to-back: host launch latency off the measured span
            HF.linear_wgrad(L.BF16, dy, x, M, N, K, bias=True)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / 10)
    ts.sort()
    print(f"{name:6s} M={M:6d} N={N:3d} K={K:3d}  median {ts[reps // 2]:6.1f} us  min {ts[0]:6.1f} us  "
          f"err dw {err:.1e} db {errb:.1e}", flush=True)
