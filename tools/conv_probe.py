"""Time hvit_conv_fwd / hvit_conv_dgrad on the default model's 3x3 convs at B=32
(bf16) against torch.nn.functional.conv2d (MIOpen, channels_last bf16) on the
same shapes: one line per conv, microseconds per launch (HIP events) and
TFLOP/s.  `fwd+bn` writes the BatchNorm tile partials as the train step does.

    python tools/conv_probe.py
"""

import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import hvit_amd_loader  # noqa: E402
from wgrad_sweep import CONVS, B  # noqa: E402

hv = hvit_amd_loader.load()
HF = sys.modules["hvit_amd.functional"]
L = hv._lib


def timeit(fn, reps=30):
    for _ in range(3):
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
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    for name, Hs, Ws, C1, C2, U, Cout, KS, S, Pd in CONVS:
        if C1 == 1 or Cout == 1 or S != 1:
            continue
        x1 = torch.randn(B, Hs, Ws, C1, device=dev).to(torch.bfloat16)
        x2 = torch.randn(B, Hs, Ws, C2, device=dev).to(torch.bfloat16) if C2 else None
        Ho, Wo = Hs * U, Ws * U
        P = B * Ho * Wo
        w = torch.randn(Cout, C1 + C2, KS, KS, device=dev) * 0.05
        wp = HF.pack_conv(w, 0, L.BF16)
        g = HF.geom(x1, C1, x2, C2, B, Hs, Ws, U, KS, S, Pd, Cout)
        z = torch.empty(B, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        tr = L.lib().hvit_conv_bn_tile_rows(g)
        part = torch.empty(((P + tr - 1) // tr, Cout, 2), device=dev)
        fl = 2.0 * P * Cout * (C1 + C2) * KS * KS
        t_bn = timeit(lambda: L.call("hvit_conv_fwd", L.BF16, g, wp.data_ptr(), None, z.data_ptr(), L.BF16,
                                     part.data_ptr(), None, s()))
        t_pl = timeit(lambda: L.call("hvit_conv_fwd", L.BF16, g, wp.data_ptr(), None, z.data_ptr(), L.BF16, None,
                                     None, s()))
        xin = x1 if x2 is None else torch.cat([x1, x2], -1)
        if U > 1:
            xin = xin.repeat_interleave(U, 1).repeat_interleave(U, 2)
        xc = xin.permute(0, 3, 1, 2)  # NCHW view of NHWC storage = channels_last
        wc = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        t_ref = timeit(lambda: F.conv2d(xc, wc, None, 1, Pd))
        wd = HF.pack_conv(w, 1, L.BF16)
        dz = torch.randn(B, Ho, Wo, Cout, device=dev).to(torch.bfloat16)
        dx = torch.empty(B, Ho, Wo, C1 + C2, device=dev, dtype=torch.bfloat16)
        t_dg = timeit(lambda: L.call("hvit_conv_dgrad", L.BF16, g, dz.data_ptr(), wd.data_ptr(), dx.data_ptr(),
                                     L.BF16, s()))
        print(f"{name:5s} fwd+bn {t_bn:7.1f} us {fl / t_bn / 1e6:5.0f} TF/s | fwd {t_pl:7.1f} us "
              f"{fl / t_pl / 1e6:5.0f} | MIOpen fwd {t_ref:7.1f} us {fl / t_ref / 1e6:5.0f} | dgrad {t_dg:7.1f} us "
              f"{fl / t_dg / 1e6:5.0f}", flush=True)


if __name__ == "__main__":
    main()
