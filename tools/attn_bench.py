"""Attention micro-benchmark at the HybridViT shape (B=32, N=256, H=8, hd=64,
bf16, attention dropout 0.1): fwd and bwd timed with HIP events."""

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


def main(p=0.1):
    B, N, H, hd = 32, 256, 8, 64
    D = H * hd
    qkv = (torch.randn(B * N, 3 * D, device="cuda") * 0.7).to(torch.bfloat16)
    o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device="cuda")
    dr = L.dropout(p, 1, 2)
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    fwd = lambda: L.call("hvit_mhsa_fwd", L.BF16, qkv.data_ptr(), B, N, H, hd, hd ** -0.5, dr, o.data_ptr(),  # noqa
                         lse.data_ptr(), None, st())
    us = timeit(fwd)
    fl = 4 * B * H * N * N * hd
    print(f"mhsa fwd p={p}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, H, N, device="cuda")
    bwd = lambda: L.call("hvit_mhsa_bwd", L.BF16, qkv.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(),  # noqa
                         B, N, H, hd, hd ** -0.5, dr, dqkv.data_ptr(), delta.data_ptr(), st())
    us = timeit(bwd)
    print(f"mhsa bwd p={p}: {us:7.1f} us  {2 * fl / us / 1e6:6.1f} TF/s", flush=True)
    if p > 0:  # keep-bit variants (the training path)
        kb = torch.empty(L.lib().hvit_mhsa_keep_bits_elems(B, N, H), dtype=torch.int32, device="cuda")
        fwdk = lambda: L.call("hvit_mhsa_fwd_kb", L.BF16, qkv.data_ptr(), B, N, H, hd, hd ** -0.5, dr,  # noqa
                              o.data_ptr(), lse.data_ptr(), kb.data_ptr(), st())
        us = timeit(fwdk)
        print(f"mhsa fwd_kb p={p}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)
        bwdk = lambda: L.call("hvit_mhsa_bwd_kb", L.BF16, qkv.data_ptr(), o.data_ptr(), do.data_ptr(),  # noqa
                              lse.data_ptr(), B, N, H, hd, hd ** -0.5, dr, kb.data_ptr(), dqkv.data_ptr(),
                              delta.data_ptr(), st())
        us = timeit(bwdk)
        print(f"mhsa bwd_kb p={p}: {us:7.1f} us  {2 * fl / us / 1e6:6.1f} TF/s", flush=True)
        rows = L.lib().hvit_mhsa_bias_rows(L.BF16, B, N, H, hd)
        parts = torch.empty(rows, 3 * D, device="cuda")
        bwdb = lambda: L.call("hvit_mhsa_bwd_db", L.BF16, qkv.data_ptr(), o.data_ptr(), do.data_ptr(),  # noqa
                              lse.data_ptr(), B, N, H, hd, hd ** -0.5, dr, kb.data_ptr(), dqkv.data_ptr(),
                              delta.data_ptr(), parts.data_ptr(), st())
        us = timeit(bwdb)
        print(f"mhsa bwd_kb+bias p={p}: {us:7.1f} us  {2 * fl / us / 1e6:6.1f} TF/s", flush=True)


def fp8_main(p=0.1):
    """config 5's attention (B=16, N=256, H=12, hd=64): the bf16 forward against
    the fp8 forms (hvit_gemm_tune(5, form): 0 round-4 kernel, 1 v2 16 waves,
    2 v2 8 waves), keep-bit entry points (the training path)."""
    B, N, H, hd = 16, 256, 12, 64
    D = H * hd
    qkv = (torch.randn(B * N, 3 * D, device="cuda") * 0.7).to(torch.bfloat16)
    o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device="cuda")
    dr = L.dropout(p, 1, 2)
    kb = torch.empty(L.lib().hvit_mhsa_keep_bits_elems(B, N, H), dtype=torch.int32, device="cuda")
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    fl = 4 * B * H * N * N * hd
    fb = lambda: L.call("hvit_mhsa_fwd_kb", L.BF16, qkv.data_ptr(), B, N, H, hd, hd ** -0.5, dr,  # noqa
                        o.data_ptr(), lse.data_ptr(), kb.data_ptr(), st())
    us = timeit(fb)
    print(f"config5 bf16 fwd_kb p={p}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)
    f8 = lambda: L.call("hvit_mhsa_fwd_fp8_kb", qkv.data_ptr(), B, N, H, hd, hd ** -0.5, dr,  # noqa
                        o.data_ptr(), lse.data_ptr(), kb.data_ptr(), st())
    old = L.lib().hvit_gemm_tune(5, 1)
    try:
        for form in (0, 1, 2):
            L.lib().hvit_gemm_tune(5, form)
            us = timeit(f8)
            print(f"config5 fp8 form {form} fwd_kb p={p}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)
    finally:
        L.lib().hvit_gemm_tune(5, old)


if __name__ == "__main__":
    if "--fp8" in sys.argv:
        fp8_main(0.1)
        fp8_main(0.0)
    else:
        main(0.1)
        main(0.0)
