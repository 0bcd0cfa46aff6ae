"""Price the long-K, N = 512 ViT GEMMs (fc1 / qkv data gradients, fc2 forward)
on larger tiles with split K: hvit_probe_gemm_splitk (f32 slabs, no
reduction) on gemm.h's kernels (cfg 0, the model's current choice) and the
gemm_ring.h configurations, graph-replayed.  The split forms' slab sum is a
separate cost (printed: one read of every slab + one f32 write at 8 TB/s).

    python tools/dgrad_split_probe.py [reps=20]
"""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib
DEV = "cuda"
BF = torch.bfloat16
M = 8192


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(ts)[2]


def main():
    args = dict(a.split("=") for a in sys.argv[1:])
    reps = int(args.get("reps", "20"))
    gen = torch.Generator(device=DEV).manual_seed(0)
    shapes = [("fc1 dgrad", 1, 0, 512, 2048), ("qkv dgrad", 1, 0, 512, 1536), ("fc2 fwd", 1, 1, 512, 2048)]
    combos = [(0, 1), (1, 1), (1, 2), (3, 1), (3, 2), (3, 4), (4, 2), (4, 4)]
    print(f"{'shape':10} {'cfg':>3} {'splits':>6} {'us':>7} {'TF/s':>6} {'+sum us':>8} {'max|d|':>9}", flush=True)
    for name, kca, kcb, N, K in shapes:
        a = (torch.randn(M, K, device=DEV, generator=gen) * 0.5).to(BF)
        b = (torch.randn(N, K, device=DEV, generator=gen) * 0.5).to(BF)
        if not kcb:
            b = b.t().contiguous()  # [K][N]
        ref = None
        for cfg, s in combos:
            ws = torch.zeros(s * (M * N + M), device=DEV)

            def go():
                L.call("hvit_probe_gemm_splitk", kca, kcb, a.data_ptr(), b.data_ptr(), M, N, K, s, ws.data_ptr(), cfg,
                       torch.cuda.current_stream().cuda_stream)

            try:
                us = timed(go, reps)
            except RuntimeError as e:
                print(f"{name:10} {cfg:>3} {s:>6}  n/a ({str(e)[:60]})", flush=True)
                continue
            c = ws.view(s, M * N + M)[:, :M * N].sum(0)
            if ref is None:
                ref = c.clone()
            d = (c - ref).abs().max().item()
            sum_us = 0.0 if s == 1 else (s + 1) * M * N * 4 / 8e12 * 1e6
            print(f"{name:10} {cfg:>3} {s:>6} {us:7.1f} {2 * M * N * K / us / 1e6:6.0f} {sum_us:8.1f} {d:9.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
