"""GPU: the train-step neighbours against plain PyTorch
fp32 references of the same ops: CombinedLoss (training/losses.py:286-387)
forward + backward, clip_grad_norm_ (trainer.py:170-174) and AdamW
(training/optimizer.py:53-61, torch.optim.AdamW), including the fused clip and
the bf16 weight shadows FusedAdamW writes."""

import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def ref_loss(pred, target, l1=1.0, mse=0.0, stoi=0.1, perc=0.0, logc=False):
    """losses.py:330-387 restated with torch ops (the reference's own formulas)."""
    pi, ti = (torch.log(pred + 1e-8), torch.log(target + 1e-8)) if logc else (pred, target)
    tot = 0.0
    if l1 > 0:
        tot = tot + l1 * F.l1_loss(pi, ti)
    if mse > 0:
        tot = tot + mse * F.mse_loss(pi, ti)
    if stoi > 0:
        pn = F.normalize(pred.flatten(1), dim=1)
        tn = F.normalize(target.flatten(1), dim=1)
        tot = tot + stoi * (1.0 - (pn * tn).sum(1)).mean()
    if perc > 0:
        tot = tot + perc * F.l1_loss(pred, target)
    return tot


CASES = [
    dict(shape=(4, 1, 64, 64), w=dict()),                                   # trainer defaults
    dict(shape=(3, 1, 33, 47), w=dict(l1=1.0, mse=0.5, stoi=0.3, perc=0.2)),  # P % 4 != 0, all terms
    dict(shape=(2, 2, 16, 20), w=dict(l1=0.7, mse=1.0, stoi=0.0, perc=0.0, logc=True)),
    dict(shape=(32, 1, 256, 256), w=dict()),                                # the bench batch
]


@pytest.mark.parametrize("case", CASES)
def test_combined_loss_fwd_bwd(hv, case):
    torch.manual_seed(1)
    shape, w = case["shape"], case["w"]
    pred = torch.rand(shape, device=DEV).requires_grad_(True)
    tgt = torch.rand(shape, device=DEV)
    ref = ref_loss(pred, tgt, **w)
    ref.backward()
    mod = hv.CombinedLoss(l1_weight=w.get("l1", 1.0), mse_weight=w.get("mse", 0.0), stoi_weight=w.get("stoi", 0.1),
                          perceptual_weight=w.get("perc", 0.0), use_log_compression=w.get("logc", False))
    p2 = pred.detach().clone().requires_grad_(True)
    out, comps = mod(p2, tgt, return_components=True)
    (2.0 * out).backward()  # upstream gradient is read on the device
    assert abs(out.item() - ref.item()) <= 1e-5 * max(1.0, abs(ref.item()))
    assert rel(p2.grad, 2.0 * pred.grad) < 1e-4
    if w.get("l1", 1.0) > 0:
        pi, ti = (torch.log(pred + 1e-8), torch.log(tgt + 1e-8)) if w.get("logc") else (pred, tgt)
        assert abs(comps["l1"].item() - F.l1_loss(pi, ti).item()) < 1e-5


def test_combined_loss_zero_prediction(hv):
    """all-zero prediction: F.normalize clamps |p| at 1e-12 (grad t / (eps |t|))."""
    pred = torch.zeros(2, 1, 8, 8, device=DEV, requires_grad=True)
    tgt = torch.rand(2, 1, 8, 8, device=DEV)
    ref_loss(pred, tgt, l1=0.0, stoi=1e-12).backward()
    p2 = pred.detach().clone().requires_grad_(True)
    hv.CombinedLoss(l1_weight=0.0, stoi_weight=1e-12)(p2, tgt).backward()
    assert rel(p2.grad, pred.grad) < 1e-4


def _params(seed, sizes=((7,), (1000,), (33, 65), (4097,), (64, 576))):
    g = torch.Generator(device="cpu").manual_seed(seed)
    ps = [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in sizes]
    return ps


def _set_grads(ps, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    for p in ps:
        p.grad = (torch.randn(p.shape, generator=g) * scale).to(DEV)


@pytest.mark.parametrize("max_norm", [0.5, 1e6])
def test_clip_grad_norm(hv, max_norm):
    a = _params(0)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    _set_grads(a, 1)
    _set_grads(b, 1)
    na = hv.clip_grad_norm_(a, max_norm)
    nb = torch.nn.utils.clip_grad_norm_(b, max_norm)
    assert abs(na.item() - nb.item()) <= 1e-5 * nb.item()
    for pa, pb in zip(a, b):
        assert rel(pa.grad, pb.grad) < 1e-5


@pytest.mark.parametrize("clip", [None, 1.0])
def test_fused_adamw_matches_torch(hv, clip):
    a = _params(2)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    oa = hv.FusedAdamW(a, lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.05, max_grad_norm=clip)
    ob = torch.optim.AdamW(b, lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.05)
    for it in range(4):
        _set_grads(a, 10 + it, scale=3.0)
        _set_grads(b, 10 + it, scale=3.0)
        oa.step()
        if clip is not None:
            torch.nn.utils.clip_grad_norm_(b, clip)
        ob.step()
    for pa, pb in zip(a, b):
        assert rel(pa.detach(), pb.detach()) < 2e-5
        assert rel(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"]) < 2e-5
        assert float(oa.state[pa]["step"]) == 4.0


def test_fused_adamw_skips_params_without_grad(hv):
    a = _params(3)
    before = [p.detach().clone() for p in a]
    opt = hv.FusedAdamW(a, lr=1e-2)
    _set_grads(a[:2], 5)
    opt.step()
    assert not torch.equal(a[0].detach(), before[0])
    for p, q in zip(a[2:], before[2:]):
        assert torch.equal(p.detach(), q) and len(opt.state[p]) == 0


def test_fused_adamw_writes_bf16_shadow(hv):
    """a bf16 forward creates the shadow; the fused step keeps it equal to bf16(p)."""
    HF = __import__("sys").modules["hvit_amd.functional"]
    torch.manual_seed(0)
    m = hv.HybridViT(encoder_channels=[8, 16, 32], embed_dim=64, num_heads=4, num_layers=1,
                     decoder_channels=[32, 16, 8, 1], precision="bf16").to(DEV).train()
    opt = hv.FusedAdamW(m.parameters(), lr=1e-3, max_grad_norm=1.0)
    x = torch.rand(2, 1, 32, 32, device=DEV)
    for _ in range(2):
        loss = hv.CombinedLoss()(m(x), x)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    w = m.transformer.blocks[0].attn.qkv.weight
    sh = HF.shadow_of(w)
    assert sh is not None and torch.equal(sh, w.detach().bfloat16())


def test_train_step_matches_torch_optimizer(hv):
    """tiny model, fp32, dropout off: 3 steps of HybridViT + CombinedLoss +
    FusedAdamW(max_grad_norm) vs the same model with torch clip + AdamW."""
    kw = dict(encoder_channels=[8, 16, 32], embed_dim=64, num_heads=4, num_layers=2, decoder_channels=[32, 16, 8, 1],
              dropout=0.0, attn_dropout=0.0, drop_path_rate=0.0, precision="fp32")
    torch.manual_seed(0)
    ma = hv.HybridViT(**kw).to(DEV).train()
    mb = copy.deepcopy(ma)
    oa = hv.FusedAdamW(ma.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    ob = torch.optim.AdamW(mb.parameters(), lr=1e-3, weight_decay=0.01)
    crit = hv.CombinedLoss()
    x = torch.rand(2, 1, 32, 48, device=DEV)
    t = torch.rand(2, 1, 32, 48, device=DEV)
    for _ in range(3):
        crit(ma(x), t).backward()
        oa.step()
        oa.zero_grad(set_to_none=True)
        crit(mb(x), t).backward()
        torch.nn.utils.clip_grad_norm_(mb.parameters(), 1.0)
        ob.step()
        ob.zero_grad(set_to_none=True)
    # Adam normalises each update to ~lr, so a parameter that starts at zero (biases)
    # carries gradient rounding differences at the scale of lr * steps: bound the
    # difference by 1e-4 of the parameter plus 1e-3 of the total update size
    for (k, pa), pb in zip(ma.named_parameters(), mb.parameters()):
        err = (pa.detach() - pb.detach()).abs().max().item()
        assert err <= 1e-4 * pb.detach().abs().max().item() + 1e-3 * 1e-3 * 3, k


def test_combined_loss_reference_fixture(hv):
    """hvit CombinedLoss against the reference's own CombinedLoss outputs
    (tests/golden/loss_cases.npz, from training/losses.py:286-387 by
    tools/gen_golden.py): loss, components and d loss / d pred."""
    import numpy as np
    from conftest import golden
    g = golden("loss_cases")
    ncase = len({k.split(".")[0] for k in g})
    for i in range(ncase):
        kw = {k.split(".")[-1]: float(v) for k, v in g.items() if k.startswith(f"c{i}.kw.")}
        if "use_log_compression" in kw:
            kw["use_log_compression"] = bool(kw["use_log_compression"])
        p = torch.as_tensor(g[f"c{i}.pred"], device=DEV).requires_grad_(True)
        loss, comps = hv.CombinedLoss(**kw)(p, torch.as_tensor(g[f"c{i}.target"], device=DEV), return_components=True)
        loss.backward()
        ref = float(g[f"c{i}.loss"])
        assert abs(loss.item() - ref) <= 1e-5 * max(1.0, abs(ref)), i
        assert rel(p.grad.cpu(), torch.as_tensor(g[f"c{i}.dpred"])) < 1e-4, i
        for k, v in comps.items():
            if k != "total":
                assert abs(v.item() - float(g[f"c{i}.comp.{k}"])) < 1e-5, (i, k)
        assert abs(comps["total"].item() - float(g[f"c{i}.comp.total"])) < 1e-5
