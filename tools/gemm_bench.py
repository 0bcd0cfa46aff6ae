"""Micro-benchmark of the libhvit GEMM family at the HybridViT B=32 shapes
(bf16), timed with HIP events on the current stream.  Prints TF/s per call."""

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


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def s():
    return torch.cuda.current_stream().cuda_stream


def report(name, flops, us):
    print(f"{name:44s} {us:9.1f} us  {flops / us / 1e6:8.1f} TF/s", flush=True)


def linear(M, N, K, tag):
    x = torch.randn(M, K, device=DEV).to(BF)
    w = torch.randn(N, K, device=DEV).to(BF)
    b = torch.zeros(N, device=DEV)
    y = torch.empty(M, N, device=DEV, dtype=BF)
    us = timeit(lambda: L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w.data_ptr(), b.data_ptr(), M, N, K,
                               y.data_ptr(), L.BF16, None, s()))
    report(f"fwd   {tag} {M}x{N}x{K}", 2 * M * N * K, us)
    dy = torch.randn(M, N, device=DEV).to(BF)
    dx = torch.empty(M, K, device=DEV, dtype=BF)
    us = timeit(lambda: L.call("hvit_linear_dgrad", L.BF16, dy.data_ptr(), w.data_ptr(), M, N, K, dx.data_ptr(),
                               L.BF16, None, s()))
    report(f"dgrad {tag}", 2 * M * N * K, us)
    us = timeit(lambda: HF.linear_wgrad(L.BF16, dy, x, M, N, K))
    report(f"wgrad {tag}", 2 * M * N * K, us)
    # library reference (hipBLASLt via torch) for the same three products
    us = timeit(lambda: torch.nn.functional.linear(x, w))
    report(f"  torch fwd   {tag}", 2 * M * N * K, us)
    us = timeit(lambda: dy @ w)
    report(f"  torch dgrad {tag}", 2 * M * N * K, us)
    us = timeit(lambda: dy.t() @ x)
    report(f"  torch wgrad {tag}", 2 * M * N * K, us)


def conv(N, Hs, Ws, C1, C2, U, Cout, tag):
    H, W = Hs * U, Ws * U
    x1 = torch.randn(N, Hs, Ws, C1, device=DEV).to(BF)
    x2 = torch.randn(N, Hs, Ws, C2, device=DEV).to(BF) if C2 else None
    w = torch.randn(Cout, C1 + C2, 3, 3, device=DEV)
    g = HF.geom(x1, C1, x2, C2, N, Hs, Ws, U, 3, 1, 1, Cout)
    wp = HF.pack_conv(w, 0, L.BF16)
    z = torch.empty(N, H, W, Cout, device=DEV, dtype=BF)
    P = N * H * W
    part = torch.empty((P + 63) // 64, Cout, 2, device=DEV)
    fl = 2 * P * Cout * 9 * (C1 + C2)
    us = timeit(lambda: L.call("hvit_conv_fwd", L.BF16, g, wp.data_ptr(), None, z.data_ptr(), L.BF16,
                               part.data_ptr(), None, s()))
    report(f"conv fwd   {tag}", fl, us)
    dz = torch.randn(N, H, W, Cout, device=DEV).to(BF)
    us = timeit(lambda: HF.conv_wgrad(L.BF16, g, dz, w.shape))
    report(f"conv wgrad {tag}", fl, us)
    if C1 > 1:
        wd = HF.pack_conv(w, 1, L.BF16)
        du = torch.empty(N, H, W, C1 + C2, device=DEV, dtype=BF)
        us = timeit(lambda: L.call("hvit_conv_dgrad", L.BF16, g, dz.data_ptr(), wd.data_ptr(), du.data_ptr(),
                                   L.BF16, s()))
        report(f"conv dgrad {tag}", fl, us)


def patch():
    N, H, W, C, D, P = 32, 64, 64, 256, 512, 4
    x = torch.randn(N, H, W, C, device=DEV).to(BF)
    w = torch.randn(D, C, P, P, device=DEV)
    g = HF.geom(x, C, None, 0, N, H, W, 1, P, P, 0, D)
    wp = HF.pack_conv(w, 0, L.BF16)
    out = torch.empty(N, 256, D, device=DEV)
    b = torch.zeros(D, device=DEV)
    fl = 2 * N * 256 * D * C * 16
    us = timeit(lambda: L.call("hvit_conv_fwd", L.BF16, g, wp.data_ptr(), b.data_ptr(), out.data_ptr(), L.F32, None,
                               None, s()))
    report("patch fwd", fl, us)
    gd = torch.randn(N * 256, D, device=DEV).to(BF)
    us = timeit(lambda: HF.conv_wgrad(L.BF16, g, gd, w.shape))
    report("patch wgrad", fl, us)
    dx = torch.empty(N, H, W, C, device=DEV, dtype=BF)
    us = timeit(lambda: L.call("hvit_conv_dgrad", L.BF16, g, gd.data_ptr(), wp.data_ptr(), dx.data_ptr(), L.BF16,
                               s()))
    report("patch dgrad", fl, us)


if __name__ == "__main__":
    torch.manual_seed(0)
    M = 32 * 256
    linear(M, 1536, 512, "qkv")
    linear(M, 512, 512, "proj")
    linear(M, 2048, 512, "fc1")
    linear(M, 512, 2048, "fc2")
    conv(32, 256, 256, 1, 0, 1, 64, "enc0")
    conv(32, 128, 128, 64, 0, 1, 128, "enc1")
    conv(32, 64, 64, 128, 0, 1, 256, "enc2")
    conv(32, 16, 16, 256, 256, 1, 256, "dec0")
    conv(32, 16, 16, 256, 128, 2, 128, "dec1")
    conv(32, 32, 32, 128, 64, 2, 64, "dec2")
    patch()
