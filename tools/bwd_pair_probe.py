"""Backward of one ViT linear (B=32 x 256 tokens, bf16): how long the data
gradient and the weight gradient take alone, back to back (the step's form:
the weight gradient's split-K slab sum carried by the data-gradient launch), and
concurrently on two streams, for several split-K workgroup targets of the
weight gradient.  HIP events on the launching stream around each form.

    python tools/bwd_pair_probe.py [reps=20] [targets=0,128,64]
"""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib
HF = sys.modules["hvit_amd.functional"]
DEV = "cuda"
BF = torch.bfloat16
M, D, HID = 8192, 512, 2048
KEEP = []


def r(*shape, dt=BF):
    t = (torch.randn(*shape, device=DEV) * 0.5).to(dt)
    KEEP.append(t)
    return t


def timeit(fn, reps):
    """``reps`` calls captured in one hipGraph (no host launch gaps, as in the
    captured step); median over 5 timed replays, per call."""
    for _ in range(3):
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
    return ts[len(ts) // 2]


def linears():
    out = []
    # name, dy [M, N], W [N, K], x [M, K], dgrad epilogue, dgrad out dtype
    gh = r(M, HID)
    cs = torch.zeros((M // 64, HID), device=DEV)
    KEEP.append(cs)
    out.append(("fc2", r(M, D), r(D, HID), r(M, HID), lambda side: HF.epilogue(act=L.ACT_MUL_AUX, aux=gh, colsum=cs,
                                                                                  side=side), L.BF16, HID))
    out.append(("fc1", r(M, HID), r(HID, D), r(M, D), lambda side: HF.epilogue(side=side), L.F32, D))
    out.append(("proj", r(M, D), r(D, D), r(M, D), lambda side: HF.epilogue(side=side), L.BF16, D))
    out.append(("qkv", r(M, 3 * D), r(3 * D, D), r(M, D), lambda side: HF.epilogue(side=side), L.F32, D))
    return out


def main():
    args = dict(a.split("=") for a in sys.argv[1:])
    reps = int(args.get("reps", "20"))
    targets = [int(t) for t in args.get("targets", "0,128,64").split(",")]
    s2 = torch.cuda.Stream()
    print(f"{'linear':6s} {'target':>6s} {'dgrad':>8s} {'wgrad+sum':>10s} {'seq(step)':>10s} {'conc w|d':>9s} "
          f"{'conc d|w':>9s}  GFLOP  TF/s(seq) TF/s(best)")
    for name, dy, W, x, epi, odt, K in linears():
        N = dy.shape[1]
        dx = torch.empty((M, K), device=DEV, dtype=torch.float32 if odt == L.F32 else BF)
        gf = 2.0 * 2 * M * N * K / 1e9

        def dgrad(side=None):
            L.call("hvit_linear_dgrad", L.BF16, dy.data_ptr(), W.data_ptr(), M, N, K, dx.data_ptr(), odt, epi(side),
                   L.stream_ptr())

        def wgrad_now():
            return HF.linear_wgrad_now(L.BF16, dy, x, M, N, K)

        def seq():
            _, j = HF.linear_wgrad_deferred(L.BF16, dy, x, M, N, K)
            dgrad(j)

        def conc(wfirst):
            def f():
                s1 = torch.cuda.current_stream()
                s2.wait_stream(s1)
                if wfirst:
                    with torch.cuda.stream(s2):
                        wgrad_now()
                    dgrad()
                else:
                    dgrad()
                    with torch.cuda.stream(s2):
                        wgrad_now()
                s1.wait_stream(s2)
            return f

        for t in targets:
            old = L.lib().hvit_gemm_tune(2, t)
            td = timeit(dgrad, reps)
            tw = timeit(wgrad_now, reps)
            ts = timeit(seq, reps)
            tc1 = timeit(conc(True), reps)
            tc2 = timeit(conc(False), reps)
            L.lib().hvit_gemm_tune(2, old)
            best = min(ts, tc1, tc2)
            print(f"{name:6s} {t:6d} {td:8.1f} {tw:10.1f} {ts:10.1f} {tc1:9.1f} {tc2:9.1f}  {gf:5.1f} "
                  f"{gf / ts * 1e3:9.0f} {gf / best * 1e3:9.0f}", flush=True)


if __name__ == "__main__":
    main()
