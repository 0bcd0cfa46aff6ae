"""Host-side (Python / ctypes) cost of one bf16 train step: cProfile over a
few steps of bench.py's step, sorted by own time.  The GPU queue is drained
before every step, so no launch blocks on a full queue and the profile shows
enqueue work only.

    python tools/host_profile.py [steps]
"""

import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
from hvit_amd.data import spectrogram_batch  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    torch.manual_seed(1234)
    model = hv.HybridViT(precision="bf16").cuda().train()
    opt = hv.FusedAdamW(model.parameters(), lr=1e-4, weight_decay=0.01, max_grad_norm=1.0)
    crit = hv.CombinedLoss()
    noisy, clean = spectrogram_batch(32, seed=1234)
    noisy, clean = noisy.cuda(), clean.cuda()

    def step():
        loss = crit(model(noisy), clean)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = 0.0
    for _ in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t += time.perf_counter() - t0
    torch.cuda.synchronize()
    print(f"host enqueue per step (queue drained first): {t / steps * 1e3:.3f} ms", flush=True)
    pr = cProfile.Profile()
    for _ in range(steps):
        torch.cuda.synchronize()
        pr.enable()
        step()
        pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
