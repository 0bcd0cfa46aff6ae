"""GPU: the reference trainer's call surface (training/trainer.py:142-205,
:350-412) driven through the build's HybridViT, CombinedLoss and FusedAdamW
(create_optimizer) exactly as Trainer.train_epoch calls them: CUDA autocast
(fp16, the reference's torch.cuda.amp default -> the bf16 HIP path),
GradScaler.scale / unscale_ / step / update, torch.nn.utils.clip_grad_norm_,
gradient accumulation, optimizer.zero_grad(), a CosineAnnealingLR scheduler,
then the Trainer checkpoint dict saved with torch.save and restored into fresh
objects, which must continue identically (to float-atomic rounding)."""

import copy
import io

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
KW = dict(encoder_channels=[8, 16, 32], embed_dim=64, num_heads=4, num_layers=2, decoder_channels=[32, 16, 8, 1])


def _objects(hv, seed=0, model=None):
    torch.manual_seed(seed)
    m = model if model is not None else hv.HybridViT(**KW).to(DEV)
    cfg = {"optimizer": {"name": "adamw", "lr": 1e-3, "weight_decay": 0.01}, "loss": {}}
    opt = hv.create_optimizer(m, cfg)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
    scaler = torch.amp.GradScaler("cuda")
    crit = hv.create_loss_function(cfg)
    return m, opt, sched, scaler, crit


def _train_steps(m, opt, sched, scaler, crit, batches, accum=2, clip=1.0):
    """trainer.py:142-183 (+ scheduler.step per epoch, :304-305)."""
    m.train()
    losses = []
    for i, (noisy, clean) in enumerate(batches):
        with torch.autocast("cuda", dtype=torch.float16):
            out = m(noisy)
            loss = crit(out, clean) / accum
        scaler.scale(loss).backward()
        if (i + 1) % accum == 0:
            scaler.unscale_(opt)
            torch.nn.utils.clip_grad_norm_(m.parameters(), clip)
            scaler.step(opt)
            scaler.update()
            opt.zero_grad()
        losses.append(loss.item() * accum)
    sched.step()
    return losses


def _batches(n, seed):
    g = torch.Generator().manual_seed(seed)
    return [(torch.rand(2, 1, 48, 64, generator=g).to(DEV), torch.rand(2, 1, 48, 64, generator=g).to(DEV))
            for _ in range(n)]


def test_trainer_loop_amp_scaler_accum_checkpoint(hv):
    m, opt, sched, scaler, crit = _objects(hv)
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    losses = _train_steps(m, opt, sched, scaler, crit, _batches(4, 1))
    assert all(torch.isfinite(torch.tensor(losses)))
    moved = [k for k, v in m.state_dict().items() if v.is_floating_point() and not torch.equal(v, before[k])]
    still = [k for k, v in m.state_dict().items() if v.is_floating_point() and k not in moved]
    assert not still, (scaler.get_scale(), still)  # every parameter and BN running statistic updated
    assert set(m.state_dict()) == set(before)
    assert all(float(opt.state[p]["step"]) == 2.0 for p in m.parameters())  # 4 micro-batches / accum 2
    assert opt.param_groups[0]["lr"] < 1e-3  # scheduler stepped

    # Trainer.save_checkpoint / load_checkpoint (trainer.py:350-412)
    ckpt = {"epoch": 0, "global_step": 2, "model_state_dict": m.state_dict(),
            "optimizer_state_dict": opt.state_dict(), "best_val_loss": 1.0, "config": {},
            "scheduler_state_dict": sched.state_dict(), "scaler_state_dict": scaler.state_dict()}
    buf = io.BytesIO()
    torch.save(ckpt, buf)
    buf.seek(0)
    ck = torch.load(buf, map_location=DEV, weights_only=True)
    m2, opt2, sched2, scaler2, crit2 = _objects(hv, seed=123)
    m2.load_state_dict(ck["model_state_dict"])
    opt2.load_state_dict(ck["optimizer_state_dict"])
    sched2.load_state_dict(ck["scheduler_state_dict"])
    scaler2.load_state_dict(ck["scaler_state_dict"])
    for p, q in zip(m.parameters(), m2.parameters()):
        for k in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(opt.state[p][k].cpu(), opt2.state[q][k].cpu())
    assert scaler2.get_scale() == scaler.get_scale()

    # both continue identically (seeded dropout: same torch seed before each;
    # float atomics in a few reductions allow last-bit differences)
    b = _batches(2, 2)
    torch.manual_seed(9)
    l1 = _train_steps(m, opt, sched, scaler, crit, b)
    torch.manual_seed(9)
    l2 = _train_steps(m2, opt2, sched2, scaler2, crit2, b)
    assert max(abs(a - c) for a, c in zip(l1, l2)) < 1e-5
    for (k, v), v2 in zip(m.state_dict().items(), m2.state_dict().values()):
        if v.is_floating_point():
            assert (v - v2).abs().max().item() <= 1e-4 * v.abs().max().item() + 1e-6, k
        else:
            assert torch.equal(v, v2), k


def test_grad_scaler_skips_step_on_inf(hv):
    """GradScaler.step (trainer.py:178) must skip FusedAdamW when unscale_
    finds an inf, and update() must back the scale off."""
    m, opt, sched, scaler, crit = _objects(hv)
    noisy, clean = _batches(1, 3)[0]
    with torch.autocast("cuda", dtype=torch.float16):
        loss = crit(m(noisy), clean)
    scaler.scale(loss).backward()
    next(m.parameters()).grad.view(-1)[0] = float("inf")
    before = [p.detach().clone() for p in m.parameters()]
    s0 = scaler.get_scale()
    scaler.unscale_(opt)
    scaler.step(opt)
    scaler.update()
    assert scaler.get_scale() < s0
    for p, q in zip(m.parameters(), before):
        assert torch.equal(p.detach(), q)
    assert all(len(opt.state[p]) == 0 for p in m.parameters())


def test_weights_only_checkpoint_roundtrip_reference_keys(hv):
    """utils/checkpoint.py:127-161 load_model_weights(strict=True): a saved
    state_dict reloads strictly with the reference's 122 keys for the default
    model, and the eval forward is unchanged."""
    m = hv.HybridViT().to(DEV).eval()
    sd = m.state_dict()
    assert len(sd) == 122
    buf = io.BytesIO()
    torch.save({"model_state_dict": sd}, buf)
    buf.seek(0)
    m2 = hv.HybridViT().to(DEV).eval()
    m2.load_state_dict(torch.load(buf, map_location=DEV, weights_only=True)["model_state_dict"], strict=True)
    x = torch.rand(1, 1, 64, 64, device=DEV)
    with torch.no_grad():
        assert torch.equal(m(x), m2(x))


def test_train_step_cuda_graph_capture(hv):
    """One whole bf16 train step (forward, CombinedLoss, backward, fused clip +
    AdamW) captured in a torch.cuda.CUDAGraph: every libhvit launch goes to the
    capturing stream with no host sync inside the step, and replays track an
    eager copy of the same model step for step."""
    kw = dict(KW, dropout=0.0, attn_dropout=0.0, drop_path_rate=0.0, precision="bf16")
    torch.manual_seed(0)
    ma = hv.HybridViT(**kw).to(DEV).train()
    mb = copy.deepcopy(ma)
    oa = hv.FusedAdamW(ma.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    ob = hv.FusedAdamW(mb.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    crit = hv.CombinedLoss()
    x, t = _batches(1, 4)[0]

    def step(m, o):
        loss = crit(m(x), t)
        loss.backward()
        o.step()
        o.zero_grad(set_to_none=True)
        return loss

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):  # warm-up: allocator pools, bf16 weight shadows, optimizer state
            step(ma, oa)
    torch.cuda.current_stream().wait_stream(side)
    for _ in range(2):
        step(mb, ob)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_loss = step(ma, oa)
    # FusedAdamW counts steps on the host (torch.optim.AdamW's bias corrections):
    # the captured launch bakes in step 3's, so compare the first replay only,
    # then check that further replays keep training
    p0 = [p.detach().clone() for p in ma.parameters()]
    g.replay()
    lb = step(mb, ob)
    torch.cuda.synchronize()
    assert abs(static_loss.item() - lb.item()) < 1e-4 * abs(lb.item())
    for (k, pa), pb in zip(ma.named_parameters(), mb.parameters()):
        assert (pa.detach() - pb.detach()).abs().max().item() <= 1e-3 * pb.detach().abs().max().item() + 1e-6, k
    l_first = static_loss.item()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    assert static_loss.item() < l_first
    assert any(not torch.equal(p.detach(), q) for p, q in zip(ma.parameters(), p0))


@pytest.mark.parametrize("kw", [KW, dict(KW, embed_dim=128, num_heads=2)], ids=["hd16", "hd64"])
def test_train_step_graph_with_dropout_and_device_counters(hv, kw):
    """The bench's graph mode: a whole bf16 train step WITH dropout (p = 0.1
    everywhere, DropPath 0.1) and FusedAdamW(capturable=True) captured once and
    replayed.  The dropout seed stream and the AdamW step counters live on the
    device, so every replay draws new masks and applies its own bias
    corrections: the parameters after each replay match an eager copy driven
    through the same number of steps from the same seed state."""
    kw = dict(kw, precision="bf16")
    torch.manual_seed(0)
    ma = hv.HybridViT(**kw).to(DEV).train()
    mb = copy.deepcopy(ma)
    oa = hv.FusedAdamW(ma.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, capturable=True)
    ob = hv.FusedAdamW(mb.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0, capturable=True)
    crit = hv.CombinedLoss()
    x, t = _batches(1, 4)[0]

    def step(m, o):
        loss = crit(m(x), t)
        loss.backward()
        o.step()
        o.zero_grad(set_to_none=True)
        return loss

    ma.set_dropout_state(12345)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            step(ma, oa)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_loss = step(ma, oa)
    mb.set_dropout_state(12345)
    for _ in range(2):
        step(mb, ob)
    losses = []
    for r in range(5):
        g.replay()
        lb = step(mb, ob)
        torch.cuda.synchronize()
        losses.append(static_loss.item())
        assert abs(static_loss.item() - lb.item()) <= 2e-3 * abs(lb.item()), (r, static_loss.item(), lb.item())
        for (k, pa), pb in zip(ma.named_parameters(), mb.parameters()):
            tol = 2e-3 * pb.detach().abs().max().item() + 1e-6
            assert (pa.detach() - pb.detach()).abs().max().item() <= tol, (r, k)
    assert len(set(losses)) == len(losses)  # every replay is a new step
    assert torch.equal(ma.dropout_state(), mb.dropout_state())
    assert int(ma.dropout_state()[1]) == 7  # 2 warm-up forwards + 5 replays (capture runs nothing)
    st = oa.state[next(ma.parameters())]["step"]
    assert st.is_cuda and float(st) == 7.0


def test_graph_replays_draw_new_dropout_masks(hv):
    """Forward-only capture in train mode (fp32): two replays give different
    outputs (new masks), equal bit for bit to two eager forwards from the same
    device seed state; two forwards before one backward keep their own masks
    (each forward's seed has its own device word)."""
    kw = dict(KW, precision="fp32")
    torch.manual_seed(1)
    m = hv.HybridViT(**kw).to(DEV).train()
    x, _ = _batches(1, 5)[0]
    m.set_dropout_state(999)
    with torch.no_grad():
        e1 = m(x).clone()
        e2 = m(x).clone()
    assert not torch.equal(e1, e2)
    m.set_dropout_state(999)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side), torch.no_grad():
        with torch.cuda.graph(g):
            y = m(x)
    torch.cuda.current_stream().wait_stream(side)
    g.replay()
    r1 = y.clone()
    g.replay()
    r2 = y.clone()
    torch.cuda.synchronize()
    assert torch.equal(r1, e1) and torch.equal(r2, e2)
    # two forwards, then one backward through both: each uses its own masks
    mb = copy.deepcopy(m)
    m.set_dropout_state(5)
    mb.set_dropout_state(5)
    xa = x.clone().requires_grad_(True)
    (m(xa).sum() + 2.0 * m(xa).sum()).backward()
    xb = x.clone().requires_grad_(True)
    mb(xb).sum().backward()
    ga = xb.grad.clone()
    xb.grad = None
    (2.0 * mb(xb).sum()).backward()
    gb = ga + xb.grad
    torch.cuda.synchronize()
    assert (xa.grad - gb).abs().max().item() <= 1e-5 * gb.abs().max().item()


def test_fused_adamw_capturable_matches_torch(hv):
    """FusedAdamW(capturable=True) step captured once, replayed 5 times with
    fresh gradients each time: device step counters give torch.optim.AdamW's
    bias corrections step by step."""
    torch.manual_seed(2)
    shapes = [(64, 32), (128,), (3, 5, 7)]
    pa = [torch.randn(s, device=DEV, requires_grad=True) for s in shapes]
    pb = [p.detach().clone().requires_grad_(True) for p in pa]
    oa = hv.FusedAdamW(pa, lr=1e-2, betas=(0.9, 0.99), weight_decay=0.05, capturable=True)
    ob = torch.optim.AdamW(pb, lr=1e-2, betas=(0.9, 0.99), weight_decay=0.05)
    grads = [[torch.randn(s, device=DEV) for s in shapes] for _ in range(7)]
    static = [torch.zeros(s, device=DEV) for s in shapes]
    for p, s in zip(pa, static):
        p.grad = s
    # one eager step (device counters created), then capture
    for s, gsrc in zip(static, grads[0]):
        s.copy_(gsrc)
    oa.step()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g):
            oa.step()
    torch.cuda.current_stream().wait_stream(side)
    for p, gsrc in zip(pb, grads[0]):
        p.grad = gsrc.clone()
    ob.step()
    for i in range(1, 6):
        for s, gsrc in zip(static, grads[i]):
            s.copy_(gsrc)
        g.replay()
        for p, gsrc in zip(pb, grads[i]):
            p.grad = gsrc.clone()
        ob.step()
        torch.cuda.synchronize()
        for a, b in zip(pa, pb):
            assert (a.detach() - b.detach()).abs().max().item() <= 2e-6 * (1 + b.detach().abs().max().item()), i
    assert float(oa.state[pa[0]]["step"]) == 6.0
    # state_dict round trip keeps counting on the device
    sd = oa.state_dict()
    oc = hv.FusedAdamW([p.detach().clone().requires_grad_(True) for p in pa], lr=1e-2, betas=(0.9, 0.99),
                       weight_decay=0.05, capturable=True)
    oc.load_state_dict(sd)
    assert float(oc.state_dict()["state"][0]["step"]) == 6.0
