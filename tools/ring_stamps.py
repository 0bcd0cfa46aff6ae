"""Where the 256x256 ring GEMM's time goes (diagnostic build libhvit_stamps.so,
-DHVIT_GEMM_STAMPS; run with HVIT_LIB=libhvit_stamps.so): per-workgroup
wall-clock stamps at start, after the K loop and at exit of
gemm_ring_kernel, for the fc1 forward (GELU dual store) and the fc2 data
gradient (GELU backward + column sums) at the B=32 ViT shape, hvit_gemm_tune(3, 0).

    HVIT_LIB=libhvit_stamps.so python tools/ring_stamps.py
"""

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pp_bench as PB  # noqa: E402
from gemm_stamps import stamps, TICK_US  # noqa: E402

L = PB.L


def report(name, fn, nblk):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = stamps(nblk)
    t0 = s[:, 0].min()
    st, k, e = (s[:, 0] - t0) * TICK_US, (s[:, 1] - s[:, 0]) * TICK_US, (s[:, 2] - s[:, 1]) * TICK_US
    end = (s[:, 2] - t0) * TICK_US
    q = lambda a: "min %5.1f med %5.1f max %5.1f" % (a.min(), np.median(a), a.max())  # noqa: E731
    print(f"{name:22s} start {q(st)} | K loop {q(k)} | epilogue {q(e)} | end {q(end)}", flush=True)
    # slot 3: wave 0's shader cycles in the per-stage vmcnt wait + barrier (diagnostic build);
    # as a share of the K loop via the in-kernel clock (cycles / wall of the same K loop)
    w = s[:, 3]
    print(f"{'':22s} K-loop wait+barrier: median {np.median(w):9.0f} cycles "
          f"(~{np.median(w) / np.median(k) / 1e3:4.2f} GHz-us of a {np.median(k):4.1f} us K loop)", flush=True)


def main():
    L.lib().hvit_gemm_tune(3, 0)
    cs = PB.cases(8192)
    for name, fl, fn, outs, tref in cs:
        if name in ("fwd fc1+gelu p0", "dgrad fc2+geluB p0", "fwd fc1+gelu p.1", "dgrad fc2+geluB p.1"):
            report(name, fn, 256)


if __name__ == "__main__":
    main()
