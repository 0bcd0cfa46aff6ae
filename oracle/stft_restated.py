"""librosa's STFT / iSTFT restated in numpy, for the host framing of the
enhancement path.

TEST INFRASTRUCTURE ONLY (see oracle/hvit_oracle.py header).

The reference frames audio with ``librosa.stft`` / ``librosa.istft``
(utils/audio_processing.py:67-98 and :101-131; inference/enhancer.py:82-89
and :111-118 with n_fft 512, hop 128, win 512, 'hann', center=True), pinned as
``librosa>=0.10.0`` (requirements.txt:9).  librosa is not installed here, so
this file restates its published 0.10 algorithm (``librosa.core.spectrum``)
step by step, as plain loops over frames:

stft:  the window is ``scipy.signal.get_window('hann', win_length,
       fftbins=True)`` (periodic), centred inside n_fft; with center=True the
       signal is padded by n_fft // 2 on both sides with ``pad_mode='constant'``
       (zeros: the 0.10 default); frame t covers padded samples
       [t * hop, t * hop + n_fft) for t < 1 + (len_padded - n_fft) // hop, and
       column t is ``rfft(window * frame)``.
istft: n_fft = 2 * (n_bins - 1); with ``length`` and center=True only the
       first ceil((length + 2 * (n_fft // 2)) / hop) frames are used; every
       frame's ``irfft(column, n_fft) * window`` is overlap-added at t * hop;
       the sum is divided by the window-square envelope
       sum_t window^2[n - t * hop] wherever that envelope exceeds the float
       tiny of its dtype (``window_sumsquare``, ``util.tiny``); center=True
       drops the first n_fft // 2 samples; the result is cut or zero-padded to
       ``length`` (``util.fix_length``).

Parity status: this is a restatement, not librosa's own output (none of the
reference's files hold STFT values), so the framing stays "parity unpinned"
against the reference; the tests check the product's torch.stft / torch.istft
framing against this restatement.
"""

from __future__ import annotations

import math
from typing import Optional

import numpy as np


def hann_periodic(win_length: int) -> np.ndarray:
    """scipy.signal.get_window('hann', win_length, fftbins=True)."""
    n = np.arange(win_length, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * math.pi * n / win_length)


def _window(n_fft: int, win_length: int) -> np.ndarray:
    w = hann_periodic(win_length)
    lpad = (n_fft - win_length) // 2  # librosa.util.pad_center
    return np.pad(w, (lpad, n_fft - win_length - lpad))


def stft(y: np.ndarray, n_fft: int = 512, hop_length: int = 128, win_length: int = 512) -> np.ndarray:
    """librosa.stft(y, n_fft, hop_length, win_length, 'hann', center=True) (0.10)."""
    y = np.asarray(y, dtype=np.float64)
    w = _window(n_fft, win_length)
    yp = np.pad(y, (n_fft // 2, n_fft // 2))  # pad_mode='constant'
    n_frames = 1 + (len(yp) - n_fft) // hop_length
    out = np.empty((n_fft // 2 + 1, n_frames), dtype=np.complex128)
    for t in range(n_frames):
        out[:, t] = np.fft.rfft(w * yp[t * hop_length:t * hop_length + n_fft])
    return out


def istft(spec: np.ndarray, hop_length: int = 128, win_length: int = 512,
          length: Optional[int] = None) -> np.ndarray:
    """librosa.istft(spec, hop_length, win_length, 'hann', center=True, length) (0.10)."""
    n_fft = 2 * (spec.shape[0] - 1)
    w = _window(n_fft, win_length)
    n_frames = spec.shape[1]
    if length is not None:
        n_frames = min(n_frames, int(math.ceil((length + 2 * (n_fft // 2)) / hop_length)))
    total = n_fft + hop_length * (n_frames - 1)
    y = np.zeros(total, dtype=np.float64)
    env = np.zeros(total, dtype=np.float64)
    for t in range(n_frames):
        s = t * hop_length
        y[s:s + n_fft] += np.fft.irfft(spec[:, t], n_fft) * w
        env[s:s + n_fft] += w * w
    nz = env > np.finfo(np.float64).tiny
    y[nz] /= env[nz]
    y = y[n_fft // 2:]
    if length is None:
        return y[:len(y) - n_fft // 2]
    if len(y) >= length:
        return y[:length]
    return np.pad(y, (0, length - len(y)))
