"""Diagnostic: where does the fp32 HIP backward depart from the oracle?
Captures the gradient w.r.t. each decoder / encoder block output and the
ViT feature map on both sides (autograd hooks on the HIP Functions' outputs,
retain_grad on the oracle's intermediates) and prints rel-L2 per tensor.
GPU + CPU oracle.  Usage: grad_trace.py CASE"""
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
HF = sys.modules["hvit_amd.functional"]
name = sys.argv[1]
g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
cfg = O.HViTConfig(**(O.TINY if name.startswith("tiny") else {}))
cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
shapes = O.state_dict_shapes(cfg)
W = CF.weights(shapes)
x = torch.as_tensor(g["x"])
t = torch.as_tensor(g["target"])

grads, outs = {}, {}
order = []


def wrap(cls, tag):
    orig = cls.apply

    def apply(*a):
        r = orig(*a)
        y = r[0] if isinstance(r, tuple) else r
        k = f"{tag}{sum(1 for o in order if o.startswith(tag))}"
        order.append(k)
        outs[k] = y.detach().float().cpu()
        y.register_hook(lambda gr, k=k: grads.__setitem__(k, gr.detach().float().cpu()))
        return r

    cls.apply = apply


wrap(HF.ConvBNActFn, "cbn")
wrap(HF.HeadFn, "head")
wrap(HF.SkipFn, "skip")
wrap(HF.FinalFn, "final")
m = hv.HybridViT(**cfg.as_kwargs(), precision="fp32").cuda()
m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
m.train()
hv.CombinedLoss()(m(x.cuda()), t.cuda()).backward()

sd = O.make_state(shapes, W, requires_grad=True)
cap = {}


class Cap(dict):
    def __setitem__(self, k, v):
        if v.requires_grad:
            v.retain_grad()
        super().__setitem__(k, v)


cap = Cap()
O.combined_loss(O.forward(sd, x, cfg, training=True, capture=cap), t).backward()
# HIP order: cbn0..2 = encoder blocks, head0 = feat, skip0..2, cbn3..5 = decoder 0..2, final0
pairs = [("cbn0", "enc0"), ("cbn1", "enc1"), ("cbn2", "enc2"), ("head0", "feat"), ("cbn3", "dec0"), ("cbn4", "dec1"),
         ("cbn5", "dec2")]


def nchw(a):
    return a.permute(0, 3, 1, 2)


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


for hk, ok in pairs:
    if hk in grads and ok in cap and cap[ok].grad is not None:
        print(f"{hk:6s}/{ok:5s} out rel {rel(nchw(outs[hk]), cap[ok].detach()):.2e}   grad rel "
              f"{rel(nchw(grads[hk]), cap[ok].grad):.2e}")
    else:
        print(hk, ok, "missing", hk in grads, ok in cap)
