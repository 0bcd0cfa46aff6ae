"""Time hvit_conv_wgrad on every conv of the default model at B=32 (bf16),
one line per conv: average microseconds over a loop of launches, measured with
HIP events on the current stream.  Planner variants are selected by the
environment of the calling process (e.g. HVIT_CONV_WG_TARGET), so a sweep runs
this once per setting:

    for t in 256 384 512; do HVIT_CONV_WG_TARGET=$t python tools/wgrad_sweep.py; done
"""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
HF = sys.modules["hvit_amd.functional"]
L = hv._lib

B = 32
# name, Hs, Ws, C1, C2, U, Cout, KS, stride, pad  (models/hybrid_vit.py:172-263 at 256x256 input)
CONVS = [
    ("enc0", 256, 256, 1, 0, 1, 64, 3, 1, 1),
    ("enc1", 128, 128, 64, 0, 1, 128, 3, 1, 1),
    ("enc2", 64, 64, 128, 0, 1, 256, 3, 1, 1),
    ("patch", 64, 64, 256, 0, 1, 512, 4, 4, 0),
    ("dec0", 16, 16, 256, 256, 1, 256, 3, 1, 1),
    ("dec1", 16, 16, 256, 128, 2, 128, 3, 1, 1),
    ("dec2", 32, 32, 128, 64, 2, 64, 3, 1, 1),
    ("dec3", 64, 64, 64, 0, 1, 1, 3, 1, 1),
]


def main(reps=30):
    dev = "cuda"
    torch.manual_seed(0)
    tot = 0.0
    for name, Hs, Ws, C1, C2, U, Cout, KS, S, Pd in CONVS:
        x1 = torch.randn(B, Hs, Ws, C1, device=dev).to(torch.bfloat16)
        x2 = torch.randn(B, Hs, Ws, C2, device=dev).to(torch.bfloat16) if C2 else None
        Ho = (Hs * U + 2 * Pd - KS) // S + 1
        Wo = (Ws * U + 2 * Pd - KS) // S + 1
        dz = torch.randn(B, Ho, Wo, Cout, device=dev).to(torch.bfloat16)
        g = HF.geom(x1, C1, x2, C2, B, Hs, Ws, U, KS, S, Pd, Cout)
        wshape = (Cout, C1 + C2, KS, KS)
        for _ in range(3):
            HF.conv_wgrad(L.BF16, g, dz, wshape)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            HF.conv_wgrad(L.BF16, g, dz, wshape)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / reps
        flop = 2.0 * B * Ho * Wo * Cout * (C1 + C2) * KS * KS
        tot += us
        print(f"{name:6s} {us:8.1f} us  {flop / us / 1e6:7.1f} TFLOP/s", flush=True)
    print(f"total  {tot:8.1f} us  [{os.environ.get('HVIT_CONV_WG_TARGET', '-')}]", flush=True)


if __name__ == "__main__":
    main()
