"""Synthetic VoiceBank-shaped spectrogram batches (host-side, no dataset).

Waveforms follow the reference notebook's synthetic generator (demo.ipynb
cell 6): f0 ~ 200 + 50 N(0,1), 7 harmonics with amplitude 1/h and random
phase, a 5 Hz envelope, peak 0.8, plus N(0, 0.15^2) noise for the noisy copy.
Spectrograms use the reference's host STFT settings (n_fft 512, hop 128,
win 512, periodic Hann, center=True; inference/enhancer.py:82-89,
data/dataset.py:183-190) and per-utterance min-max scaling
(data/dataset.py:213-219).  STFT/iSTFT stay on the host (north star).
"""

from __future__ import annotations

import numpy as np
import torch

SR = 16000
N_FFT, HOP, WIN = 512, 128, 512


def harmonic_pair(n_samples: int, seed: int):
    rng = np.random.Generator(np.random.PCG64(seed))
    t = np.arange(n_samples) / SR
    f0 = 200.0 + 50.0 * rng.standard_normal()
    clean = np.zeros(n_samples)
    for h in range(1, 8):
        clean += (1.0 / h) * np.sin(2 * np.pi * f0 * h * t + rng.random() * 2 * np.pi)
    clean *= 0.5 + 0.5 * np.sin(2 * np.pi * 5 * t)
    clean = clean / np.abs(clean).max() * 0.8
    noisy = clean + 0.15 * rng.standard_normal(n_samples)
    return clean.astype(np.float32), noisy.astype(np.float32)


def magnitude(wave: np.ndarray) -> torch.Tensor:
    x = torch.as_tensor(wave)
    spec = torch.stft(x, N_FFT, HOP, WIN, window=torch.hann_window(WIN), center=True, pad_mode="constant",
                      return_complex=True)
    return spec.abs()


def minmax(m: torch.Tensor) -> torch.Tensor:
    lo, hi = m.min(), m.max()
    return (m - lo) / (hi - lo) if hi > lo else m


def spectrogram_batch(batch: int, freq: int = 256, frames: int = 256, seed: int = 1234):
    """(noisy, clean) magnitude batches [B, 1, freq, frames] in [0, 1]."""
    n = (frames - 1) * HOP
    noisy, clean = [], []
    for i in range(batch):
        c, nz = harmonic_pair(n, seed + i)
        noisy.append(minmax(magnitude(nz))[:freq, :frames])
        clean.append(minmax(magnitude(c))[:freq, :frames])
    return torch.stack(noisy)[:, None].contiguous(), torch.stack(clean)[:, None].contiguous()
