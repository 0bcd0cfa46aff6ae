"""Generate the golden parity fixtures under tests/golden/ (build container only).

This script imports the reference's own ``models`` package and its
``training/losses.py`` (loaded by file path, so ``training/__init__``'s
tensorboard import is never executed) from /root/reference (read-only;
PYTHONDONTWRITEBYTECODE=1) and records their outputs on inputs/weights from
``oracle/closed_form.py``.  It is never run on the GPU box and nothing else in
the repository imports the reference.  The fixtures are plain ``.npz`` data
(inputs, expected outputs, intermediates, gradients).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py [name ...]
"""

import importlib.util
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True
REF = "/root/reference"
sys.path.insert(0, REF)

from models.hybrid_vit import HybridViT  # noqa: E402  (the reference)

from oracle import closed_form as CF  # noqa: E402
from oracle import hvit_oracle as O  # noqa: E402


def _ref_losses():
    spec = importlib.util.spec_from_file_location("ref_training_losses", os.path.join(REF, "training", "losses.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


RL = _ref_losses()  # training/losses.py: CombinedLoss :286-387, STOILoss :88-141

OUT = os.path.join(ROOT, "tests", "golden")
LARGE = dict(embed_dim=768, num_heads=12, num_layers=12)   # BASELINE config 5 dims


def build(cfgkw, train):
    kw = O.HViTConfig(**cfgkw)
    if train:
        kw.dropout = kw.attn_dropout = kw.drop_path_rate = 0.0
    m = HybridViT(**kw.as_kwargs())
    W = CF.weights(O.state_dict_shapes(kw))
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()})
    return m, kw


def hooks(m, store):
    hs = []
    for i, blk in enumerate(m.encoder):
        hs.append(blk.register_forward_hook(lambda mod, a, o, i=i: store.__setitem__(f"enc{i}", o)))
    hs.append(m.patch_embed.register_forward_hook(lambda mod, a, o: store.__setitem__("tokens", o[0])))
    hs.append(m.transformer.register_forward_hook(
        lambda mod, a, o: store.__setitem__("vit_out", o[0] if isinstance(o, tuple) else o)))
    last = m.decoder[-1].block[0 if m.decoder[-1].block[0].__class__.__name__ == "Conv2d" else 1]
    hs.append(last.register_forward_hook(lambda mod, a, o: store.__setitem__("pre_tanh", o)))
    return hs


def record(name, cfgkw, shape, seed, full_grads=True, with_attn=True,
           keep=("enc0", "enc1", "enc2", "tokens", "vit_out", "pre_tanh"), full16=(), rows16=None):
    """full16: parameter names whose full gradient is stored as float16
    (``full16.<name>``; ``rows16`` limits a name to its first rows)."""
    x = torch.as_tensor(CF.spectrogram(shape, seed))
    tgt = torch.as_tensor(CF.spectrogram(shape, seed + 1000))
    d = {"x": x.numpy(), "target": tgt.numpy()}
    # ---- eval forward (+ attentions) ----
    m, kw = build(cfgkw, train=False)
    m.eval()
    st = {}
    hs = hooks(m, st)
    with torch.no_grad():
        if with_attn:
            y, attn = m(x, return_attentions=True)
            for l, a in enumerate(attn):
                d[f"eval_attn{l}"] = a.numpy()
        else:
            y = m(x)
    for h in hs:
        h.remove()
    d["eval_out"] = y.numpy()
    for k, v in st.items():
        if k in keep:
            d[f"eval_{k}"] = v.detach().numpy()
    # ---- train-mode step (dropout / attn dropout / drop path = 0) ----
    m, kw = build(cfgkw, train=True)
    m.train()
    st = {}
    hs = hooks(m, st)
    y = m(x)
    for h in hs:
        h.remove()
    loss = RL.CombinedLoss()(y, tgt)     # the reference's own loss (create_loss_function defaults)
    loss.backward()
    d["train_out"] = y.detach().numpy()
    d["train_loss"] = np.float64(loss.item())
    d["train_pre_tanh"] = st["pre_tanh"].detach().numpy()
    N = st["tokens"].shape[1] + (1 if m.cls_token is not None else 0)   # positional rows used
    rows16 = rows16 or {}
    for k, p in m.named_parameters():
        g = p.grad.detach()
        d[f"gnorm.{k}"] = np.float64(g.double().norm().item())
        if k == "pos_encoding.pos_embed":
            g = g[:, :N]
        if full_grads or g.numel() <= 4096:
            d[f"grad.{k}"] = g.numpy()
        if k in full16:
            g16 = g[: rows16[k]] if k in rows16 else g
            d[f"full16.{k}"] = g16.numpy().astype(np.float16)
    for k, b in m.named_buffers():
        if "running" in k:
            d[f"buf.{k}"] = b.numpy()
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **d)
    print(f"{path}: {os.path.getsize(path) / 1e6:.2f} MB, N={N}, loss={loss.item():.6f}")


LOSS_CASES = [  # CombinedLoss kwargs (training/losses.py:295-302); case 0 = create_loss_function defaults
    dict(),
    dict(l1_weight=0.5, mse_weight=0.7, stoi_weight=0.3, perceptual_weight=0.2),
    dict(l1_weight=1.0, mse_weight=0.25, stoi_weight=0.1, use_log_compression=True),
    dict(l1_weight=0.0, mse_weight=1.0, stoi_weight=0.0),
]


def record_losses():
    """The reference CombinedLoss (forward value, components, d loss / d pred)
    on tanh-range predictions and [0, 1) targets, several weight settings."""
    d = {}
    for i, kw in enumerate(LOSS_CASES):
        shape = (3, 1, 40, 56)
        pred = torch.as_tensor(2.0 * CF.spectrogram(shape, 300 + i) - 1.0)
        if kw.get("use_log_compression"):
            pred = pred.abs() + 0.05      # log(x + eps) needs positive predictions
        tgt = torch.as_tensor(CF.spectrogram(shape, 400 + i))
        p = pred.clone().requires_grad_(True)
        loss, comps = RL.CombinedLoss(**kw)(p, tgt, return_components=True)
        loss.backward()
        d[f"c{i}.pred"] = pred.numpy()
        d[f"c{i}.target"] = tgt.numpy()
        d[f"c{i}.loss"] = np.float64(loss.item())
        d[f"c{i}.dpred"] = p.grad.numpy()
        for k, v in comps.items():
            d[f"c{i}.comp.{k}"] = np.float64(v)
        for k, v in kw.items():
            d[f"c{i}.kw.{k}"] = np.float64(v)
    path = os.path.join(OUT, "loss_cases.npz")
    np.savez_compressed(path, **d)
    print(f"{path}: {os.path.getsize(path) / 1e6:.2f} MB")


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.manual_seed(0)
    want = set(sys.argv[1:])
    jobs = {
        "tiny_64": lambda: record("tiny_64", O.TINY, (2, 1, 64, 64), 11),
        "tiny_odd": lambda: record("tiny_odd", O.TINY, (1, 1, 33, 47), 12),
        "tiny_clip": lambda: record("tiny_clip", O.TINY, (1, 1, 257, 251), 13, with_attn=False,
                                    keep=("enc2", "tokens", "vit_out", "pre_tanh")),
        "default_256": lambda: record(
            "default_256", {}, (2, 1, 256, 256), 14, full_grads=False, with_attn=False, keep=("vit_out", "pre_tanh"),
            full16=("transformer.blocks.5.attn.qkv.weight", "transformer.blocks.5.attn.proj.weight",
                    "patch_embed.projection.weight"),
            rows16={"patch_embed.projection.weight": 64}),
        "default_clip": lambda: record("default_clip", {}, (1, 1, 257, 251), 15, full_grads=False, with_attn=False,
                                       keep=("pre_tanh",)),
        # BASELINE config 5 architecture (D=768, 12 heads, 12 layers)
        "large_256": lambda: record("large_256", LARGE, (1, 1, 256, 256), 16, full_grads=False, with_attn=False,
                                    keep=("vit_out", "pre_tanh")),
        # use_cls_token=True (hybrid_vit.py:118-123, 323-338; never set by create_hybrid_vit)
        "tiny_cls": lambda: record("tiny_cls", dict(O.TINY, use_cls_token=True), (2, 1, 48, 80), 17),
        "loss_cases": record_losses,
    }
    for name, job in jobs.items():
        if not want or name in want:
            job()


if __name__ == "__main__":
    main()
