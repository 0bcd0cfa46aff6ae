"""Time the attention kernels (hvit_mhsa_fwd / hvit_mhsa_bwd, bf16) on the
default model's shape (B=32, 8 heads, N=256, head dim 64) with and without
attention dropout, to separate the softmax / MFMA work from the dropout hash.

    python tools/attn_sweep.py
"""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


def main():
    dev = "cuda"
    B, N, H, hd = int(os.environ.get("ATTN_B", "32")), 256, 8, 64
    D = H * hd
    torch.manual_seed(0)
    s = torch.cuda.current_stream().cuda_stream
    qkv = (torch.randn(B * N, 3 * D, device=dev) * 0.5).to(torch.bfloat16)
    o = torch.empty(B * N, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=dev)
    do = torch.randn(B * N, D, device=dev).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, H, N, device=dev)
    flop = 4.0 * B * H * N * N * hd
    for p in (0.0, 0.1):
        dr = L.dropout(p, 77, 5)
        tf = timeit(lambda: L.call("hvit_mhsa_fwd", L.BF16, qkv.data_ptr(), B, N, H, hd, hd ** -0.5, dr,
                                   o.data_ptr(), lse.data_ptr(), None, s))
        tb = timeit(lambda: L.call("hvit_mhsa_bwd", L.BF16, qkv.data_ptr(), o.data_ptr(), do.data_ptr(),
                                   lse.data_ptr(), B, N, H, hd, hd ** -0.5, dr, dqkv.data_ptr(), delta.data_ptr(), s))
        print(f"p={p}: fwd {tf:6.1f} us {flop / tf / 1e6:5.0f} TF/s | bwd {tb:6.1f} us "
              f"{2 * flop / tb / 1e6:5.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
