"""Enhancement CLI (the reference's enhance.py, SURVEY §3.C: a working
replacement for its broken one), BASELINE config 1.

    python enhance.py --checkpoint best_model.pth --input noisy.wav --output enhanced.wav
    python enhance.py --checkpoint best_model.pth --input-dir noisy/ --output-dir enhanced/ --extension .wav
    python enhance.py --synthetic 2.0 --output enhanced.wav     # 2 s harmonic clip, no checkpoint

The reference's flags (enhance.py:26-86) with its meaning: ``--config-dir``
(default ``config``) is merged by ``load_all_configs`` (data / model / train
YAMLs, utils/config.py:77-110); an unreadable directory falls back to the
defaults with a warning (enhance.py:105-110); its ``model`` section feeds
``create_hybrid_vit`` and its ``audio`` section the enhancer's STFT settings
(:131-138); ``--extension`` picks the files of directory mode (:160-165).
Additions: ``--config`` (one more YAML merged on top), ``--synthetic``,
``--precision``.  STFT / iSTFT on the host; the HybridViT forward on the GPU
(HIP path, fp32 unless --precision bf16).
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser(description="Enhance noisy audio with the HybridViT (MI355X HIP path)")
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--config-dir", default="config", help="directory of data/model/train_config.yaml")
    ap.add_argument("--config", default=None, help="one more YAML merged on top of --config-dir's")
    ap.add_argument("--input", default=None)
    ap.add_argument("--output", default=None)
    ap.add_argument("--input-dir", default=None)
    ap.add_argument("--output-dir", default=None)
    ap.add_argument("--extension", default=".wav", help="audio file extension (directory mode)")
    ap.add_argument("--synthetic", type=float, default=None, help="seconds of synthetic noisy audio")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--no-normalize", action="store_true")
    a = ap.parse_args(argv)
    single = a.input is not None and a.output is not None
    directory = a.input_dir is not None and a.output_dir is not None
    if a.synthetic is None and not single and not directory:
        ap.error("Must specify either:\n  --input and --output for single file mode, or\n"
                 "  --input-dir and --output-dir for directory mode")
    if single and directory:
        ap.error("Cannot use both single file and directory mode simultaneously")

    import torch
    import hvit_amd_loader

    hv = hvit_amd_loader.load()
    from hvit_amd import enhancer as E

    try:
        cfg = hv.load_all_configs(a.config_dir)
    except Exception:  # the reference's bare except (enhance.py:106-110)
        print("Warning: Could not load config files. Using defaults.")
        cfg = {}
    if a.config:
        cfg = hv.merge_configs(cfg, hv.load_config(a.config) or {})
    model = hv.create_hybrid_vit(cfg, precision=a.precision)
    if a.checkpoint:
        model = E.load_model_for_inference(a.checkpoint, model, a.device)
    elif a.synthetic is None:
        ap.error("--checkpoint is required unless --synthetic is given")
    au = cfg.get("audio", {}) or {}
    enh = E.AudioEnhancer(model, device=a.device, sample_rate=au.get("sample_rate", 16000), n_fft=au.get("n_fft", 512),
                          hop_length=au.get("hop_length", 128), win_length=au.get("win_length", 512))
    norm = not a.no_normalize
    if a.synthetic is not None:
        torch.manual_seed(0)
        clip = E.synthetic_clip(a.synthetic)
        out = enh.enhance(clip, normalize=norm)
        print(f"synthetic {a.synthetic:.2f} s clip: {len(clip)} samples -> {len(out)} samples, "
              f"rms in {float((clip ** 2).mean() ** 0.5):.4f} out {float((out ** 2).mean() ** 0.5):.4f}")
        if a.output:
            E.write_wav(a.output, out, enh.sample_rate)
    elif single:
        enh.enhance_file(a.input, a.output, normalize=norm)
    else:
        enh.enhance_directory(a.input_dir, a.output_dir, extension=a.extension, normalize=norm)


if __name__ == "__main__":
    main()
