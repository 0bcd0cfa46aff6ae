"""What bounds the ViT weight gradients (B=32 x 256 tokens, bf16): the
split-K GEMM dW[N, K] = dy^T x timed alone (graph replay, per call) for each
operand layout -- token-major [M][N] / [M][K] as the model holds dy and x
(the weight gradient reads them M/N-contiguous: kc = 0), or pre-transposed
K-contiguous copies (kc = 1: what a producer writing dy^T / x^T would give) --
each pipeline (gemm.h, ring 128x128 / 256x128 / 256x256) and split count, plus
the slab sum that completes the gradient.

    python tools/wgrad_layout_probe.py [reps=20]
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
MT, D, HID = 8192, 512, 2048  # token rows, model width, MLP width


def timeit(fn, reps):
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
    ts.sort()
    return ts[2]


def main():
    args = dict(a.split("=") for a in sys.argv[1:])
    reps = int(args.get("reps", "20"))
    torch.manual_seed(0)
    # name, dW rows (N_out), dW cols (K_in)
    shapes = [("fc2", D, HID), ("fc1", HID, D), ("qkv", 3 * D, D), ("proj", D, D)]
    print(f"{'wgrad':5s} {'layout':7s} {'cfg':>3s} {'splits':>6s} {'gemm us':>8s} {'sum us':>7s} {'total':>7s} "
          f"{'TF/s':>6s}  check")
    for name, n, k in shapes:
        dy = (torch.randn(MT, n, device=DEV) * 0.5).to(BF)  # token-major, as the model holds them
        x = (torch.randn(MT, k, device=DEV) * 0.5).to(BF)
        dyT, xT = dy.t().contiguous(), x.t().contiguous()  # K(token)-contiguous copies
        ref = (dy.float().t() @ x.float())
        gf = 2.0 * MT * n * k / 1e9
        for kc in (0, 1):
            a, b = (dyT, xT) if kc else (dy, x)
            for cfg in (0, 2, 3, 4):
                for splits in (1, 2, 4, 8, 16):
                    ws = torch.empty(splits * (n * k + n), device=DEV)
                    out = torch.empty(n, k, device=DEV)

                    def gemm():
                        return L.lib().hvit_probe_gemm_splitk(kc, kc, a.data_ptr(), b.data_ptr(), n, k, MT, splits,
                                                                ws.data_ptr(), cfg, L.stream_ptr())

                    if gemm() != 0:
                        L.lib().hvit_last_error()
                        continue

                    def ssum():
                        L.call("hvit_sum_slabs_strided", ws.data_ptr(), splits, n * k + n, n * k, out.data_ptr(),
                               L.stream_ptr())

                    torch.cuda.synchronize()
                    if splits > 1:
                        ssum()
                        got = out
                    else:
                        got = ws[:n * k].view(n, k)
                    torch.cuda.synchronize()
                    err = ((got - ref).abs().max() / ref.abs().max()).item()
                    tg = timeit(gemm, reps)
                    tsum = timeit(ssum, reps) if splits > 1 else 0.0
                    lay = "tok-maj" if kc == 0 else "K-contig"
                    print(f"{name:5s} {lay:7s} {cfg:3d} {splits:6d} {tg:8.1f} {tsum:7.1f} {tg + tsum:7.1f} "
                          f"{gf / (tg + tsum) * 1e3:6.0f}  {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
