"""Diagnostic: relative L2 error of every parameter gradient of one fp32 train
step against a golden fixture (tests/golden), printed worst first.  GPU only."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import hvit_amd_loader  # noqa: E402
from oracle import closed_form as CF  # noqa: E402
from oracle import hvit_oracle as O  # noqa: E402

hv = hvit_amd_loader.load()
name = sys.argv[1] if len(sys.argv) > 1 else "default_clip"
g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
cfg = O.HViTConfig(**(O.TINY if name.startswith("tiny") else {}))
cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
W = CF.weights(O.state_dict_shapes(cfg))
m = hv.HybridViT(**cfg.as_kwargs(), precision="fp32").cuda()
m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
m.train()
y = m(torch.as_tensor(g["x"]).cuda())
loss = hv.CombinedLoss()(y, torch.as_tensor(g["target"]).cuda())
loss.backward()
torch.cuda.synchronize()
print("loss", loss.item(), float(g["train_loss"]))
rows = []
for k, p in m.named_parameters():
    gk = f"grad.{k}"
    if gk not in g:
        continue
    got = p.grad.detach().cpu().double()
    ref = torch.as_tensor(g[gk]).double()
    if k == "pos_encoding.pos_embed":
        got = got[:, : ref.shape[1]]
    rows.append(((got - ref).norm().item() / max(ref.norm().item(), 1e-30), k))
for r, k in sorted(rows, reverse=True):
    print(f"{r:.3e}  {k}")
