"""Reference point for the ViT linear GEMMs: torch.matmul (hipBLASLt) vs the
hvit GEMM on the same bf16 shapes (B=32 x 256 tokens), forward (x W^T),
dgrad (dy W) and wgrad (dy^T x).  Plain products only: no bias / activation
epilogues on either side.  Prints microseconds and TFLOP/s per shape.

    python tools/gemm_ref.py
"""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib

M = 8192
SHAPES = [("qkv", 1536, 512), ("proj", 512, 512), ("fc1", 2048, 512), ("fc2", 512, 2048)]  # (N_out, K_in)


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
    torch.manual_seed(0)
    s = torch.cuda.current_stream().cuda_stream
    for name, N, K in SHAPES:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * M * N * K
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        b = torch.zeros(N, device=dev)
        t_ref = timeit(lambda: torch.matmul(x, w.t()))
        t_hv = timeit(lambda: L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w.data_ptr(), b.data_ptr(), M, N, K,
                                     y.data_ptr(), L.BF16, None, s))
        t_ref_d = timeit(lambda: torch.matmul(dy, w))
        t_ref_w = timeit(lambda: torch.matmul(dy.t(), x))
        print(f"{name:5s} fwd: hipBLASLt {t_ref:7.1f} us {flop / t_ref / 1e6:6.0f} TF/s | hvit {t_hv:7.1f} us "
              f"{flop / t_hv / 1e6:6.0f} TF/s || dgrad hipBLASLt {t_ref_d:7.1f} us {flop / t_ref_d / 1e6:6.0f} TF/s"
              f" | wgrad hipBLASLt {t_ref_w:7.1f} us {flop / t_ref_w / 1e6:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
