"""GPU: BASELINE config 1 plumbing -- a synthetic 2 s clip through the
enhancer (host STFT, HybridViT on the HIP path, host iSTFT) against the same
enhancer around the CPU oracle forward."""

import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import closed_form as CF
from oracle import hvit_oracle as O

pytestmark = pytest.mark.gpu


class OracleModel(nn.Module):
    def __init__(self, sd, cfg):
        super().__init__()
        self.sd, self.cfg = sd, cfg

    def forward(self, x):
        return O.forward(self.sd, x.cpu(), self.cfg, training=False)


def test_enhance_clip_matches_oracle(hv):
    from hvit_amd import enhancer as E

    cfg = O.HViTConfig(**O.TINY)
    shapes = O.state_dict_shapes(cfg)
    W = CF.weights(shapes)
    m = hv.HybridViT(**cfg.as_kwargs(), precision="fp32")
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    clip = E.synthetic_clip(2.0, seed=5)
    out = E.AudioEnhancer(m, device="cuda").enhance(clip)
    ref = E.AudioEnhancer(OracleModel(O.make_state(shapes, W), cfg), device="cpu").enhance(clip)
    assert out.shape == clip.shape
    assert np.abs(out - ref).max() < 2e-3 * np.abs(ref).max()


def test_enhance_cli(hv, tmp_path):
    """enhance.py (BASELINE config 1's CLI) end to end on the GPU: a YAML model
    config, a Trainer-style checkpoint dict, --input/--output, --input-dir/
    --output-dir and --synthetic; the files it writes equal the in-process
    AudioEnhancer's output for the same weights."""
    import yaml

    import enhance
    from hvit_amd import enhancer as E

    cfg = {"model": {"encoder": {"channels": [8, 16, 32]},
                     "transformer": {"embed_dim": 64, "num_heads": 4, "num_layers": 2},
                     "decoder": {"channels": [32, 16, 8, 1]}}}
    (tmp_path / "cfg.yaml").write_text(yaml.safe_dump(cfg))
    ocfg = O.HViTConfig(**O.TINY)
    W = CF.weights(O.state_dict_shapes(ocfg))
    m = hv.create_hybrid_vit(cfg, precision="fp32")
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    ck = tmp_path / "best_model.pth"
    torch.save({"epoch": 1, "model_state_dict": m.state_dict(), "best_val_loss": 0.1}, ck)  # trainer.py:350-380
    d_in, d_out = tmp_path / "in", tmp_path / "out"
    d_in.mkdir()
    clips = [E.synthetic_clip(0.6, seed=20 + i) for i in range(2)]
    for i, c in enumerate(clips):
        E.write_wav(d_in / f"n{i}.wav", c, 16000)
    ref = E.AudioEnhancer(m.cuda().eval(), device="cuda")
    common = ["--checkpoint", str(ck), "--config", str(tmp_path / "cfg.yaml")]
    enhance.main(common + ["--input", str(d_in / "n0.wav"), "--output", str(tmp_path / "e0.wav")])
    got = E.read_wav(tmp_path / "e0.wav", 16000)
    want = ref.enhance(E.read_wav(d_in / "n0.wav", 16000))
    assert got.shape == clips[0].shape
    assert np.abs(got - want).max() < 1e-4 * max(np.abs(want).max(), 1e-6) + 1e-4
    enhance.main(common + ["--input-dir", str(d_in), "--output-dir", str(d_out)])
    for i in range(2):
        got = E.read_wav(d_out / f"n{i}.wav", 16000)
        want = ref.enhance(E.read_wav(d_in / f"n{i}.wav", 16000))
        assert np.abs(got - want).max() < 1e-4 * max(np.abs(want).max(), 1e-6) + 1e-4
    enhance.main(["--config", str(tmp_path / "cfg.yaml"), "--synthetic", "0.5", "--output", str(tmp_path / "s.wav")])
    s = E.read_wav(tmp_path / "s.wav", 16000)
    assert s.shape == (8000,) and np.isfinite(s).all()
    with pytest.raises(SystemExit):
        enhance.main(["--config", str(tmp_path / "cfg.yaml")])


def test_enhance_cli_reference_flags(hv, tmp_path):
    """The reference's own command line (enhance.py:26-86) on a directory of
    WAVs, as a subprocess: --checkpoint, --config-dir (three YAMLs merged by
    load_all_configs: the model section of model_config.yaml, an audio section
    overridden by a later file), --input-dir / --output-dir, --extension,
    --device.  Only files with the extension are enhanced; each output equals
    the in-process AudioEnhancer's for the same weights."""
    import subprocess
    import sys

    import yaml

    from hvit_amd import enhancer as E

    cdir = tmp_path / "config"
    cdir.mkdir()
    model = {"encoder": {"channels": [8, 16, 32]}, "transformer": {"embed_dim": 64, "num_heads": 4, "num_layers": 2},
             "decoder": {"channels": [32, 16, 8, 1]}}
    (cdir / "data_config.yaml").write_text(yaml.safe_dump({"audio": {"sample_rate": 16000, "n_fft": 512}}))
    (cdir / "model_config.yaml").write_text(yaml.safe_dump({"model": model, "audio": {"hop_length": 128}}))
    (cdir / "train_config.yaml").write_text(yaml.safe_dump({"training": {"batch_size": 16}}))
    ocfg = O.HViTConfig(**O.TINY)
    W = CF.weights(O.state_dict_shapes(ocfg))
    m = hv.create_hybrid_vit({"model": model}, precision="fp32")
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    ck = tmp_path / "best_model.pth"
    torch.save({"epoch": 3, "model_state_dict": m.state_dict()}, ck)
    d_in, d_out = tmp_path / "noisy", tmp_path / "enhanced"
    d_in.mkdir()
    clips = [E.synthetic_clip(0.5 + 0.1 * i, seed=40 + i) for i in range(2)]
    for i, c in enumerate(clips):
        E.write_wav(d_in / f"u{i}.wav", c, 16000)
    E.write_wav(d_in / "other.wv", clips[0], 16000)  # not the extension: skipped
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "enhance.py"), "--checkpoint", str(ck), "--config-dir",
                        str(cdir), "--input-dir", str(d_in), "--output-dir", str(d_out), "--extension", ".wav",
                        "--device", "cuda"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sorted(p.name for p in d_out.iterdir()) == ["u0.wav", "u1.wav"]
    ref = E.AudioEnhancer(m.cuda().eval(), device="cuda")
    for i in range(2):
        got = E.read_wav(d_out / f"u{i}.wav", 16000)
        want = ref.enhance(E.read_wav(d_in / f"u{i}.wav", 16000))
        assert got.shape == clips[i].shape
        assert np.abs(got - want).max() < 1e-4 * max(np.abs(want).max(), 1e-6) + 1e-4
