"""Audio enhancement around the HybridViT hot path (BASELINE
config 1): the reference's ``AudioEnhancer`` (inference/enhancer.py:15-290)
with the same call surface -- ``enhance``, ``enhance_file``,
``enhance_directory``, ``enhance_audio``, ``enhance_file`` (module level) and
``load_model_for_inference``.

STFT / iSTFT framing stays on the host, as the north star says.  librosa is
not available here, so the framing is ``torch.stft`` / ``torch.istft`` with the
reference's settings (n_fft 512, hop 128, win 512, periodic Hann,
center=True, constant padding -- librosa >= 0.10's ``pad_mode`` default;
enhancer.py:82-89, :111-118).  tests/test_enhancer.py checks both against a
numpy restatement of librosa 0.10's algorithm (oracle/stft_restated.py; an
inconsistent spectrum for the iSTFT, ragged lengths); against librosa's own
output the framing stays parity unpinned.  WAV I/O uses
``scipy.io.wavfile`` (soundfile is absent); files at another sample rate are
refused rather than resampled.  The model call itself is the HIP path.
"""

from __future__ import annotations

from pathlib import Path
from typing import Union

import numpy as np
import torch
import torch.nn as nn


def _window(win_length: int, window: str) -> torch.Tensor:
    if window != "hann":
        raise NotImplementedError(f"hvit enhancer: window {window!r} (the reference uses 'hann')")
    return torch.hann_window(win_length, dtype=torch.float64)  # periodic, like librosa's get_window


class AudioEnhancer:
    """inference/enhancer.py:15-56 (constructor) and :57-135 (enhance)."""

    def __init__(self, model: nn.Module, device: str = "cuda", sample_rate: int = 16000, n_fft: int = 512,
                 hop_length: int = 128, win_length: int = 512, window: str = "hann"):
        self.model = model.to(device).eval()
        self.device = device
        self.sample_rate = sample_rate
        self.n_fft = n_fft
        self.hop_length = hop_length
        self.win_length = win_length
        self.window = window

    def stft(self, audio: np.ndarray) -> torch.Tensor:
        x = torch.as_tensor(np.asarray(audio, dtype=np.float64))
        return torch.stft(x, self.n_fft, self.hop_length, self.win_length, window=_window(self.win_length, self.window),
                          center=True, pad_mode="constant", return_complex=True)

    def istft(self, spec: torch.Tensor, length: int) -> np.ndarray:
        y = torch.istft(spec, self.n_fft, self.hop_length, self.win_length,
                        window=_window(self.win_length, self.window), center=True, length=length)
        return y.numpy()

    @torch.no_grad()
    def enhance(self, noisy_audio: np.ndarray, normalize: bool = True) -> np.ndarray:
        noisy_audio = np.asarray(noisy_audio, dtype=np.float32)
        max_val = 1.0
        if normalize:
            mv = float(np.abs(noisy_audio).max()) if noisy_audio.size else 0.0
            if mv > 1e-8:
                noisy_audio = noisy_audio / mv
                max_val = mv
        spec = self.stft(noisy_audio)
        mag, phase = spec.abs(), spec.angle()
        mag_max = float(mag.max())
        if mag_max > 1e-8:
            mag_n = mag / mag_max
        else:
            mag_n, mag_max = mag, 1.0
        x = mag_n.float()[None, None].to(self.device)  # [1, 1, F, T]
        enh = self.model(x).squeeze().double().cpu() * mag_max
        out = self.istft(torch.polar(enh, phase), len(noisy_audio))
        if normalize:
            out = out * max_val
        return out.astype(np.float32)

    def enhance_file(self, input_path: Union[str, Path], output_path: Union[str, Path],
                     normalize: bool = True) -> None:
        audio = read_wav(input_path, self.sample_rate)
        out = self.enhance(audio, normalize=normalize)
        output_path = Path(output_path)
        output_path.parent.mkdir(parents=True, exist_ok=True)
        write_wav(output_path, out, self.sample_rate)
        print(f"Enhanced audio saved to {output_path}")

    def enhance_directory(self, input_dir: Union[str, Path], output_dir: Union[str, Path], extension: str = ".wav",
                          normalize: bool = True) -> None:
        files = sorted(Path(input_dir).glob(f"*{extension}"))
        Path(output_dir).mkdir(parents=True, exist_ok=True)
        print(f"Found {len(files)} audio files to enhance")
        for f in files:
            self.enhance_file(f, Path(output_dir) / f.name, normalize=normalize)
        print(f"All files enhanced and saved to {output_dir}")


def read_wav(path: Union[str, Path], sample_rate: int) -> np.ndarray:
    """Mono float32 in [-1, 1] (the reference's librosa.load(sr, mono=True),
    without resampling: a different rate is an error)."""
    from scipy.io import wavfile

    sr, data = wavfile.read(str(path))
    if sr != sample_rate:
        raise ValueError(f"hvit enhancer: {path} is {sr} Hz, expected {sample_rate} (no resampler here)")
    if np.issubdtype(data.dtype, np.integer):
        data = data.astype(np.float32) / float(np.iinfo(data.dtype).max + 1)
    data = data.astype(np.float32)
    return data.mean(axis=1) if data.ndim == 2 else data


def write_wav(path: Union[str, Path], audio: np.ndarray, sample_rate: int) -> None:
    from scipy.io import wavfile

    wavfile.write(str(path), sample_rate, np.asarray(audio, dtype=np.float32))


def enhance_audio(noisy_audio: np.ndarray, model: nn.Module, device: str = "cuda", sample_rate: int = 16000,
                  n_fft: int = 512, hop_length: int = 128) -> np.ndarray:
    """enhancer.py:198-226."""
    return AudioEnhancer(model, device, sample_rate, n_fft, hop_length).enhance(noisy_audio)


def enhance_file(input_path, output_path, model: nn.Module, device: str = "cuda", sample_rate: int = 16000) -> None:
    """enhancer.py:229-255."""
    AudioEnhancer(model, device, sample_rate).enhance_file(input_path, output_path)


def load_model_for_inference(checkpoint_path: Union[str, Path], model: nn.Module, device: str = "cuda",
                             strict: bool = True) -> nn.Module:
    """enhancer.py:258-290 with a loader that executes nothing from the file
    (weights_only=True): a Trainer checkpoint dict (``model_state_dict``,
    trainer.py:350-380) or a bare state_dict."""
    ckpt = torch.load(str(checkpoint_path), map_location="cpu", weights_only=True)
    sd = ckpt["model_state_dict"] if isinstance(ckpt, dict) and "model_state_dict" in ckpt else ckpt
    model.load_state_dict(sd, strict=strict)
    return model.to(device).eval()


def synthetic_clip(seconds: float = 2.0, seed: int = 0, sample_rate: int = 16000) -> np.ndarray:
    """A noisy harmonic clip (data.harmonic_pair) for plumbing checks (config 1)."""
    from .data import harmonic_pair

    return harmonic_pair(int(round(seconds * sample_rate)), seed)[1]


__all__ = ["AudioEnhancer", "enhance_audio", "enhance_file", "load_model_for_inference", "read_wav", "write_wav",
           "synthetic_clip"]
