"""CPU: the host side of the enhancement path (BASELINE
config 1): STFT -> magnitude normalisation -> model -> iSTFT with the noisy
phase (inference/enhancer.py:57-135), WAV I/O, checkpoint loading
(enhancer.py:258-290).  The model is a stand-in here (identity), so no GPU
work runs; tests/test_gpu_enhancer.py runs the HybridViT itself."""

import numpy as np
import pytest
import torch
import torch.nn as nn


class Identity(nn.Module):
    def forward(self, x):
        return x


def test_identity_model_reconstructs_audio(hv):
    from hvit_amd import enhancer as E

    clip = E.synthetic_clip(0.5, seed=3)
    enh = E.AudioEnhancer(Identity(), device="cpu")
    out = enh.enhance(clip)
    assert out.shape == clip.shape and out.dtype == np.float32
    assert np.abs(out - clip).max() < 1e-5 * np.abs(clip).max()
    out2 = enh.enhance(clip, normalize=False)
    assert np.abs(out2 - clip).max() < 1e-5 * np.abs(clip).max()


def test_spectrogram_shape_matches_reference_settings(hv):
    from hvit_amd import enhancer as E

    enh = E.AudioEnhancer(Identity(), device="cpu")
    spec = enh.stft(np.zeros(32000, dtype=np.float32))
    assert tuple(spec.shape) == (257, 251)  # 2 s at 16 kHz: the config-1 clip [1, 1, 257, 251]


def test_silence_is_passed_through(hv):
    from hvit_amd import enhancer as E

    out = E.AudioEnhancer(Identity(), device="cpu").enhance(np.zeros(4000, dtype=np.float32))
    assert np.all(out == 0)


def test_wav_round_trip(hv, tmp_path):
    from hvit_amd import enhancer as E

    clip = E.synthetic_clip(0.25, seed=1)
    p = tmp_path / "a.wav"
    E.write_wav(p, clip, 16000)
    assert np.array_equal(E.read_wav(p, 16000), clip)
    with pytest.raises(ValueError):
        E.read_wav(p, 8000)


def test_enhance_file_and_directory(hv, tmp_path):
    from hvit_amd import enhancer as E

    d_in, d_out = tmp_path / "in", tmp_path / "out"
    d_in.mkdir()
    for i in range(2):
        E.write_wav(d_in / f"n{i}.wav", E.synthetic_clip(0.2, seed=i), 16000)
    E.AudioEnhancer(Identity(), device="cpu").enhance_directory(d_in, d_out)
    for i in range(2):
        a = E.read_wav(d_out / f"n{i}.wav", 16000)
        b = E.read_wav(d_in / f"n{i}.wav", 16000)
        assert np.abs(a - b).max() < 1e-5


def test_load_model_for_inference_trainer_checkpoint(hv, tmp_path):
    from hvit_amd import enhancer as E

    kw = dict(encoder_channels=[8, 16, 32], embed_dim=64, num_heads=4, num_layers=2, decoder_channels=[32, 16, 8, 1])
    torch.manual_seed(0)
    src = hv.HybridViT(**kw)
    ck = tmp_path / "best_model.pth"
    torch.save({"epoch": 3, "model_state_dict": src.state_dict(), "best_val_loss": 0.5}, ck)  # trainer.py:350-380
    dst = E.load_model_for_inference(ck, hv.HybridViT(**kw), device="cpu")
    assert not dst.training
    for (k, a), b in zip(src.state_dict().items(), dst.state_dict().values()):
        assert torch.equal(a, b), k
    torch.save(src.state_dict(), tmp_path / "bare.pth")
    E.load_model_for_inference(tmp_path / "bare.pth", hv.HybridViT(**kw), device="cpu")


# ---- the host framing against librosa 0.10's algorithm, restated -------------
# (oracle/stft_restated.py; librosa itself is absent, so this pins the product's
# torch.stft / torch.istft calls against the published algorithm, not against
# librosa's output: the framing stays "parity unpinned" against the reference)

@pytest.mark.parametrize("n", [32000, 4001, 511, 300])
def test_stft_matches_restated_librosa(hv, n):
    from hvit_amd import data as Dt
    from hvit_amd import enhancer as E
    from oracle import stft_restated as R

    y = np.random.Generator(np.random.PCG64(n)).standard_normal(n).astype(np.float32)
    ref = R.stft(y)
    got = E.AudioEnhancer(Identity(), device="cpu").stft(y).numpy()
    assert got.shape == ref.shape
    tol = 1e-10 * np.abs(ref).max()
    assert np.abs(got - ref).max() <= tol
    # the training-data path (data.magnitude, f32) frames the same way
    mag = Dt.magnitude(y).numpy()
    assert mag.shape == ref.shape
    assert np.abs(mag - np.abs(ref)).max() <= 2e-5 * np.abs(ref).max()


@pytest.mark.parametrize("n", [32000, 4001, 700])
def test_istft_matches_restated_librosa(hv, n):
    from hvit_amd import enhancer as E
    from oracle import stft_restated as R

    rng = np.random.Generator(np.random.PCG64(7 + n))
    frames = 1 + n // 128
    # an arbitrary (inconsistent) spectrum: exercises the overlap-add and the
    # window-square normalisation, not just the analysis / synthesis round trip
    spec = rng.standard_normal((257, frames)) + 1j * rng.standard_normal((257, frames))
    spec[0].imag = 0.0
    spec[-1].imag = 0.0
    ref = R.istft(spec, length=n)
    got = E.AudioEnhancer(Identity(), device="cpu").istft(torch.as_tensor(spec), n)
    assert got.shape == ref.shape == (n,)
    assert np.abs(got - ref).max() <= 1e-10 * np.abs(ref).max()


def test_load_all_configs_merge_order(hv, tmp_path, capsys):
    """load_all_configs (utils/config.py:77-110): data, model, train YAMLs in
    that order, nested dicts merged key by key, a later file's keys winning;
    a missing file is reported and skipped; a missing directory raises."""
    import yaml

    (tmp_path / "data_config.yaml").write_text(yaml.safe_dump({"audio": {"sample_rate": 16000, "n_fft": 512},
                                                                "data": {"a": 1}}))
    (tmp_path / "model_config.yaml").write_text(yaml.safe_dump({"audio": {"n_fft": 1024, "hop_length": 256},
                                                                 "model": {"transformer": {"embed_dim": 64}}}))
    cfg = hv.load_all_configs(tmp_path)
    assert cfg == {"audio": {"sample_rate": 16000, "n_fft": 1024, "hop_length": 256}, "data": {"a": 1},
                   "model": {"transformer": {"embed_dim": 64}}}
    assert "train_config.yaml" in capsys.readouterr().out
    with pytest.raises(FileNotFoundError):
        hv.load_all_configs(tmp_path / "absent")
    base = {"x": {"y": 1}}
    assert hv.merge_configs(base, {"x": {"z": 2}}) == {"x": {"y": 1, "z": 2}} and base == {"x": {"y": 1}}


def test_enhance_cli_argument_errors(hv):
    """enhance.py keeps the reference's mode checks (enhance.py:90-103)."""
    import enhance

    with pytest.raises(SystemExit):
        enhance.main(["--checkpoint", "x.pth"])  # neither mode
    with pytest.raises(SystemExit):
        enhance.main(["--checkpoint", "x.pth", "--input", "a.wav", "--output", "b.wav", "--input-dir", "i",
                      "--output-dir", "o"])  # both modes
