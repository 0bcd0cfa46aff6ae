"""GEMM scaling probe: bf16 linear_fwd TF/s as K grows (steady-state loop
efficiency vs prologue/epilogue overhead), plus the torch (hipBLASLt) figure."""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import hvit_amd_loader  # noqa: E402
from gemm_bench import timeit  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib
BF = torch.bfloat16


def run(M, N, K):
    x = torch.randn(M, K, device="cuda").to(BF)
    w = torch.randn(N, K, device="cuda").to(BF)
    b = torch.zeros(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=BF)
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    us = timeit(lambda: L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w.data_ptr(), b.data_ptr(), M, N, K,
                               y.data_ptr(), L.BF16, None, st()))
    ut = timeit(lambda: torch.nn.functional.linear(x, w))
    f = 2 * M * N * K
    print(f"M={M:6d} N={N:5d} K={K:5d}  hvit {us:8.1f} us {f / us / 1e6:7.1f} TF   torch {ut:8.1f} us "
          f"{f / ut / 1e6:7.1f} TF", flush=True)


if __name__ == "__main__":
    for K in (512, 1024, 2048, 4096, 8192):
        run(8192, 2048, K)
    for K in (512, 2048, 8192):
        run(8192, 512, K)
    run(4096, 4096, 4096)
    run(8192, 8192, 8192)
