"""Diagnostic: dump forward intermediates and all parameter gradients of one
fp32 train step (golden fixture inputs) to gpurun_out/<tag>.npz, for A/B
comparisons of two library builds (HVIT_LIB).  GPU only."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import hvit_amd_loader  # noqa: E402
from oracle import closed_form as CF  # noqa: E402
from oracle import hvit_oracle as O  # noqa: E402

hv = hvit_amd_loader.load()
name, tag = sys.argv[1], sys.argv[2]
g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
cfg = O.HViTConfig(**(O.TINY if name.startswith("tiny") else {}))
cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
W = CF.weights(O.state_dict_shapes(cfg))
m = hv.HybridViT(**cfg.as_kwargs(), precision="fp32").cuda()
m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
m.train()
x = torch.as_tensor(g["x"]).cuda()
if len(sys.argv) > 3:  # relative input perturbation (sensitivity probe)
    x = x * (1 + float(sys.argv[3]) * torch.randn(x.shape, generator=torch.Generator().manual_seed(0)).cuda())
out = {}
with torch.no_grad():
    h, skips = m.forward_encoder(x)
    for i, s in enumerate(skips):
        out[f"enc{i}"] = s.float().cpu().numpy()
y = m(x)
out["y"] = y.detach().cpu().numpy()
loss = hv.CombinedLoss()(y, torch.as_tensor(g["target"]).cuda())
loss.backward()
for k, p in m.named_parameters():
    if p.numel() <= 600_000:  # small tensors only (the box returns <= 64 MiB)
        out["grad." + k] = p.grad.detach().cpu().numpy()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", tag + ".npz"), **out)
print("ok", tag)
