"""Attribute small aten launches (fills, copies, elementwise) in one bench
train step to their Python call sites (torch.profiler with stacks).  GPU only;
diagnostic, not part of the product."""
import os
import sys
from collections import Counter

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
from hvit_amd.data import spectrogram_batch  # noqa: E402

torch.manual_seed(0)
model = hv.HybridViT(precision="bf16").cuda().train()
opt = hv.FusedAdamW(model.parameters(), lr=1e-4, weight_decay=0.01, max_grad_norm=1.0)  # bench.py's step
crit = hv.CombinedLoss()
x, t = spectrogram_batch(32, seed=1)
x, t = x.cuda(), t.cuda()


def step():
    y = model(x)
    loss = crit(y, t)
    loss.backward()
    opt.step()  # clip to 1.0 + AdamW
    opt.zero_grad(set_to_none=True)


for _ in range(3):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
keys = ("fill_", "zero_", "zeros", "copy_", "clone", "add", "mul", "empty_strided", "to", "contiguous", "cat", "stack")
cnt = Counter()
for ev in prof.events():
    if ev.name.startswith("aten::") and any(k in ev.name for k in ("fill_", "zero_", "copy_", "clone", "add_", "add",
                                                                        "mul", "cat", "stack", "where", "div")):
        st = [s for s in (ev.stack or []) if "site-packages" not in s and "<built-in" not in s][:3]
        cnt[(ev.name, " <- ".join(st))] += 1
for (name, st), n in sorted(cnt.items(), key=lambda kv: -kv[1]):
    print(f"{n:4d}  {name:28s} {st}")
