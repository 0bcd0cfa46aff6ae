"""Generate the golden parity fixtures under tests/golden/ (build container only).

This script imports the reference's own ``models`` package from
/root/reference (read-only; PYTHONDONTWRITEBYTECODE=1) and records its outputs
on inputs/weights from ``oracle/closed_form.py``.  It is never run on the GPU
box and nothing else in the repository imports the reference.  The fixtures are
plain ``.npz`` data (inputs, expected outputs, intermediates, gradients).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py
"""

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference")

from models.hybrid_vit import HybridViT  # noqa: E402  (the reference)

from oracle import closed_form as CF  # noqa: E402
from oracle import hvit_oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


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
           keep=("enc0", "enc1", "enc2", "tokens", "vit_out", "pre_tanh")):
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
    loss = O.combined_loss(y, tgt)   # == CombinedLoss(l1=1, stoi=0.1), losses.py:330-387
    loss.backward()
    d["train_out"] = y.detach().numpy()
    d["train_loss"] = np.float64(loss.item())
    d["train_pre_tanh"] = st["pre_tanh"].detach().numpy()
    N = st["tokens"].shape[1]
    for k, p in m.named_parameters():
        g = p.grad.detach()
        d[f"gnorm.{k}"] = np.float64(g.double().norm().item())
        if k == "pos_encoding.pos_embed":
            g = g[:, :N]
        if full_grads or g.numel() <= 4096:
            d[f"grad.{k}"] = g.numpy()
    for k, b in m.named_buffers():
        if "running" in k:
            d[f"buf.{k}"] = b.numpy()
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **d)
    print(f"{path}: {os.path.getsize(path) / 1e6:.2f} MB, N={N}, loss={loss.item():.6f}")


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.manual_seed(0)
    record("tiny_64", O.TINY, (2, 1, 64, 64), 11)
    record("tiny_odd", O.TINY, (1, 1, 33, 47), 12)
    record("tiny_clip", O.TINY, (1, 1, 257, 251), 13, with_attn=False,
           keep=("enc2", "tokens", "vit_out", "pre_tanh"))
    record("default_256", {}, (2, 1, 256, 256), 14, full_grads=False, with_attn=False,
           keep=("vit_out", "pre_tanh"))
    record("default_clip", {}, (1, 1, 257, 251), 15, full_grads=False, with_attn=False,
           keep=("pre_tanh",))


if __name__ == "__main__":
    main()
