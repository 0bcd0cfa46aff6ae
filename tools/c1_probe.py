"""Isolated timing of the fused first-block kernels at the model's enc0 shape
(B=32, 256x256, Cout=64, pool 2, bf16): hvit_c1block_stats / _fwd / _bwd.
Usage: python tools/c1_probe.py [reps=20] [mfma=1]  (also the workload of the
rocprofv3 --pmc passes in tools/pmc_c1.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib
HF = sys.modules["hvit_amd.functional"]
args = dict(a.split("=") for a in sys.argv[1:])
reps = int(args.get("reps", 20))
L.lib().hvit_gemm_tune(1, int(args.get("mfma", 1)))
N, H, W, C, P = int(args.get("n", 32)), 256, 256, 64, 2
dev = "cuda"
x = torch.rand(N, H, W, 1, device=dev).to(torch.bfloat16)
w = torch.randn(C, 1, 3, 3, device=dev) / 3
wp = HF.pack_conv(w, 0, L.BF16)
g = HF.geom(x, 1, None, 0, N, H, W, 1, 3, 1, 1, C)
tr = L.lib().hvit_conv_bn_tile_rows(g)
part = torch.empty(((N * H * W + tr - 1) // tr, C, 2), device=dev)
mean, inv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
y = torch.empty(N, H // P, W // P, C, device=dev, dtype=torch.bfloat16)
dy = torch.randn_like(y)
sums = torch.zeros(L.lib().hvit_bn_act_bwd_sums_elems(C), device=dev)
dwp = torch.empty(C * 9, device=dev)
ws_n = L.lib().hvit_c1block_bwd_ws(g, P)
ws = torch.empty(ws_n, device=dev)
dr = L.dropout(0.1, 5, 100)
s = torch.cuda.current_stream().cuda_stream


def stats():
    L.call("hvit_c1block_stats", L.BF16, g, wp.data_ptr(), part.data_ptr(), s)


def fwd():
    L.call("hvit_c1block_fwd", L.BF16, g, wp.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(),
           beta.data_ptr(), dr, P, y.data_ptr(), L.BF16, s)


def bwd():
    L.call("hvit_c1block_bwd", L.BF16, g, wp.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(),
           beta.data_ptr(), dr, P, dy.data_ptr(), L.BF16, 1, sums.data_ptr(), 0, dwp.data_ptr(), ws.data_ptr(), ws_n,
           s)


for name, fn in (("stats", stats), ("fwd", fwd), ("bwd", bwd)):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):  # back-to-back: host launch latency off the measured span
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / 10)
    ts.sort()
    print(f"{name:6s} median {ts[len(ts) // 2]:8.1f} us  min {ts[0]:8.1f} us", flush=True)
