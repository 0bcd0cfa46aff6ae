"""GPU: variable-length batches through the per-shape graph cache
(…_amd/train_step.py; data/dataset.py:297-347 pads T per
batch).  A bf16 HybridViT with dropout trained through GraphedTrainStep on a
sequence of batches of three different T (with an LRU cap of two graphs, so a
shape's graph is evicted and captured again) equals, bit for bit after every
step, an identical copy trained eagerly from the same dropout seed state."""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
KW = dict(encoder_channels=[8, 16, 32], embed_dim=128, num_heads=2, num_layers=2, decoder_channels=[32, 16, 8, 1],
          precision="bf16")


def test_graph_cache_variable_length_matches_eager(hv):
    import importlib

    ts = importlib.import_module("hvit_amd.train_step")
    torch.manual_seed(0)
    ma = hv.HybridViT(**KW).to(DEV).train()
    mb = copy.deepcopy(ma)
    oa = hv.FusedAdamW(ma.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, capturable=True)
    ob = hv.FusedAdamW(mb.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, capturable=True)
    crit = hv.CombinedLoss()
    step = ts.GraphedTrainStep(ma, crit, oa, max_graphs=2, warmup=1)
    ma.set_dropout_state(31337)
    mb.set_dropout_state(31337)
    g = torch.Generator().manual_seed(3)
    Ts = [64, 64, 64, 48, 48, 48, 64, 80, 80, 80, 64, 64, 48, 48]
    for i, T in enumerate(Ts):
        x = torch.rand(2, 1, 48, T, generator=g).to(DEV)
        t = torch.rand(2, 1, 48, T, generator=g).to(DEV)
        la = step(x, t)
        lb = crit(mb(x), t)
        lb.backward()
        ob.step()
        ob.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        assert la.item() == lb.item(), (i, T, la.item(), lb.item())
        for (k, pa), pb in zip(ma.named_parameters(), mb.parameters()):
            assert torch.equal(pa.detach(), pb.detach()), (i, T, k)
    assert step.captures >= 4  # 64, 48, 80, and 64 again after its eviction (cap 2)
    assert step.replays >= 6
    assert len(step.cache) <= 2
    assert torch.equal(ma.dropout_state(), mb.dropout_state())


def test_graph_cache_follows_lr_scheduler(hv):
    """a replayed optimizer step must use the learning rate an
    LR scheduler set after the capture (the reference trainer steps
    CosineAnnealingLR, trainer.py:304-309).  FusedAdamW(capturable) reads
    lr / betas / eps / weight_decay on the device (sync_hyper); the graphed
    model stays bit-identical to an eager copy whose scheduler steps the same."""
    import importlib

    ts = importlib.import_module("hvit_amd.train_step")
    torch.manual_seed(1)
    ma = hv.HybridViT(**KW).to(DEV).train()
    mb = copy.deepcopy(ma)
    oa = hv.FusedAdamW(ma.parameters(), lr=2e-3, weight_decay=0.05, max_grad_norm=1.0, capturable=True)
    ob = hv.FusedAdamW(mb.parameters(), lr=2e-3, weight_decay=0.05, max_grad_norm=1.0, capturable=True)
    sa = torch.optim.lr_scheduler.CosineAnnealingLR(oa, T_max=4, eta_min=1e-5)
    sb = torch.optim.lr_scheduler.CosineAnnealingLR(ob, T_max=4, eta_min=1e-5)
    crit = hv.CombinedLoss()
    step = ts.GraphedTrainStep(ma, crit, oa, warmup=1)
    ma.set_dropout_state(99)
    mb.set_dropout_state(99)
    g = torch.Generator().manual_seed(5)
    lrs = []
    for i in range(7):
        x = torch.rand(2, 1, 48, 64, generator=g).to(DEV)
        t = torch.rand(2, 1, 48, 64, generator=g).to(DEV)
        la = step(x, t)
        lb = crit(mb(x), t)
        lb.backward()
        ob.step()
        ob.zero_grad(set_to_none=True)
        sa.step()
        sb.step()
        # a weight-decay change between replays as well (param_groups edited by hand)
        if i == 4:
            for o in (oa, ob):
                o.param_groups[0]["weight_decay"] = 0.0
        torch.cuda.synchronize()
        lrs.append(oa.param_groups[0]["lr"])
        assert la.item() == lb.item(), (i, la.item(), lb.item())
        for (k, pa), pb in zip(ma.named_parameters(), mb.parameters()):
            assert torch.equal(pa.detach(), pb.detach()), (i, k)
    assert step.captures == 1 and step.replays >= 5
    assert len(set(lrs)) >= 4  # the schedule really moved between replays
