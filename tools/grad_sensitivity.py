"""Diagnostic: how well-conditioned are the fp32 parameter gradients of a
golden case?  Prints, per parameter group, the relative-L2 distance between
  hip  vs oracle            (the parity error),
  hip(x) vs hip(x + 1e-7 x noise)        (the build's own conditioning),
  oracle(x) vs oracle(x + 1e-7 x noise)  (the reference math's conditioning).
GPU + CPU oracle.  Usage: grad_sensitivity.py CASE [eps]"""
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
name = sys.argv[1]
eps = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-7
g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
cfg = O.HViTConfig(**(O.TINY if name.startswith("tiny") else {}))
cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
shapes = O.state_dict_shapes(cfg)
W = CF.weights(shapes)
x0 = torch.as_tensor(g["x"])
t = torch.as_tensor(g["target"])
x1 = x0 * (1 + eps * torch.randn(x0.shape, generator=torch.Generator().manual_seed(0)))


def hip(x):
    m = hv.HybridViT(**cfg.as_kwargs(), precision="fp32").cuda()
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    m.train()
    hv.CombinedLoss()(m(x.cuda()), t.cuda()).backward()
    return {k: p.grad.detach().cpu().double() for k, p in m.named_parameters()}


def orc(x):
    sd = O.make_state(shapes, W, requires_grad=True)
    O.combined_loss(O.forward(sd, x, cfg, training=True), t).backward()
    return {k: v.grad.double() for k, v in sd.items() if v.grad is not None}


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


H0, H1, R0, R1 = hip(x0), hip(x1), orc(x0), orc(x1)
H0b = hip(x0)
print("per-parameter (backward order): hip-vs-oracle  hip-repeat  hip-sensitivity")
for k in list(H0)[::-1]:
    print(f"  {k:50s} {rel(H0[k], R0[k]):.2e} {rel(H0b[k], H0[k]):.2e} {rel(H1[k], H0[k]):.2e}")
groups = {}
for k in H0:
    grp = k.split(".")[0] + ("" if not k.startswith("transformer") else "." + ".".join(k.split(".")[3:]))
    r = groups.setdefault(grp, [0.0, 0.0, 0.0])
    r[0] = max(r[0], rel(H0[k], R0[k]))
    r[1] = max(r[1], rel(H1[k], H0[k]))
    r[2] = max(r[2], rel(R1[k], R0[k]))
print(f"{name} eps={eps}: group  hip-vs-oracle  hip-sensitivity  oracle-sensitivity")
for grp, (a, b, c) in sorted(groups.items(), key=lambda kv: -kv[1][0]):
    print(f"  {grp:40s} {a:.2e} {b:.2e} {c:.2e}")
