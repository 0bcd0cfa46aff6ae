"""Time the BatchNorm -> ReLU -> Dropout2d -> MaxPool backward (hvit_bn_act_bwd:
reduce pass + apply pass) on every BN layer of the default model at B=32
(bf16, training), one line per layer: average microseconds over a loop of
calls (HIP events on the current stream) and the algorithmic bytes rate.

    python tools/bn_sweep.py          # run under rocprofv3 for per-kernel times
"""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib

B = int(os.environ.get("BN_SWEEP_B", "32"))
# name, H, W, C, pool (conv output grid of each ConvBlock / TransposeConvBlock at 256x256 input)
LAYERS = [
    ("enc0", 256, 256, 64, 2),
    ("enc1", 128, 128, 128, 2),
    ("enc2", 64, 64, 256, 1),
    ("dec0", 16, 16, 256, 1),
    ("dec1", 32, 32, 128, 1),
    ("dec2", 64, 64, 64, 1),
]


def main(reps=30):
    dev = "cuda"
    torch.manual_seed(0)
    lib = L.lib()
    s = torch.cuda.current_stream().cuda_stream
    tot = 0.0
    only = os.environ.get("BN_SWEEP_ONLY")
    for name, H, W, C, P in LAYERS:
        if only and name not in only.split(","):
            continue
        z = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(B, H // P, W // P, C, device=dev).to(torch.bfloat16)
        dz = torch.empty_like(z)
        mean = torch.randn(C, device=dev) * 0.1
        invstd = torch.rand(C, device=dev) + 0.5
        gamma = torch.rand(C, device=dev) + 0.5
        beta = torch.randn(C, device=dev) * 0.1
        sums = torch.zeros(lib.hvit_bn_act_bwd_sums_elems(C), device=dev)
        drop = L.dropout(0.1, 1234, 7)

        def run():
            L.call("hvit_bn_act_bwd", L.BF16, z.data_ptr(), B, H, W, C, mean.data_ptr(), invstd.data_ptr(),
                   gamma.data_ptr(), beta.data_ptr(), drop, P, dy.data_ptr(), L.BF16, 1,
                   dz.data_ptr(), L.BF16, sums.data_ptr(), 0, s)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / reps
        nbytes = 2 * z.numel() * 2 + 2 * dy.numel() * 2 + dz.numel() * 2  # two passes over z, dy; dz once
        tot += us
        print(f"{name:5s} {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)
    print(f"total {tot:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
