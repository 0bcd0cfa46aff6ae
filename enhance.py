"""Enhancement CLI (the reference's enhance.py, SURVEY §3.C: a working
replacement for its broken one), BASELINE config 1.

    python enhance.py --checkpoint best_model.pth --input noisy.wav --output enhanced.wav
    python enhance.py --checkpoint best_model.pth --input-dir noisy/ --output-dir enhanced/
    python enhance.py --synthetic 2.0 --output enhanced.wav     # 2 s harmonic clip, no checkpoint

STFT / iSTFT on the host; the HybridViT forward on the GPU (HIP path, fp32
unless --precision bf16).  --config takes a YAML with a ``model`` section
(create_hybrid_vit keys); without it the default architecture is used.
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser(description="Enhance noisy audio with the HybridViT (MI355X HIP path)")
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--config", default=None, help="YAML file with a 'model' section")
    ap.add_argument("--input", default=None)
    ap.add_argument("--output", default=None)
    ap.add_argument("--input-dir", default=None)
    ap.add_argument("--output-dir", default=None)
    ap.add_argument("--synthetic", type=float, default=None, help="seconds of synthetic noisy audio")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--no-normalize", action="store_true")
    a = ap.parse_args(argv)

    import torch
    import hvit_amd_loader

    hv = hvit_amd_loader.load()
    from hvit_amd import enhancer as E

    cfg = {}
    if a.config:
        import yaml

        with open(a.config) as f:
            cfg = yaml.safe_load(f) or {}
    model = hv.create_hybrid_vit(cfg, precision=a.precision)
    if a.checkpoint:
        model = E.load_model_for_inference(a.checkpoint, model, a.device)
    elif a.synthetic is None:
        ap.error("--checkpoint is required unless --synthetic is given")
    enh = E.AudioEnhancer(model, device=a.device)
    norm = not a.no_normalize
    if a.synthetic is not None:
        torch.manual_seed(0)
        clip = E.synthetic_clip(a.synthetic)
        out = enh.enhance(clip, normalize=norm)
        print(f"synthetic {a.synthetic:.2f} s clip: {len(clip)} samples -> {len(out)} samples, "
              f"rms in {float((clip ** 2).mean() ** 0.5):.4f} out {float((out ** 2).mean() ** 0.5):.4f}")
        if a.output:
            E.write_wav(a.output, out, enh.sample_rate)
    elif a.input and a.output:
        enh.enhance_file(a.input, a.output, normalize=norm)
    elif a.input_dir and a.output_dir:
        enh.enhance_directory(a.input_dir, a.output_dir, normalize=norm)
    else:
        ap.error("give --input/--output, --input-dir/--output-dir or --synthetic")


if __name__ == "__main__":
    main()
