"""GPU: the whole HybridViT forward/backward on libhvit.so against the golden
vectors recorded from the reference (tests/golden, via tools/gen_golden.py) and
against the CPU oracle.  North-star bar: fp32 forward within 1e-3 relative of
the reference; bf16 path within bf16 tolerances."""

import os

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import closed_form as CF
from oracle import hvit_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

FP32_TOL = 1e-3      # north_star: forward within 1e-3 rel (fp32)
BF16_TOL = 5e-2
LARGE = dict(embed_dim=768, num_heads=12, num_layers=12)   # BASELINE config 5 architecture


def grad_tol(name, key):
    """Relative-L2 bar for a parameter gradient of a whole-model train step.

    fp32 gradients of the 28M-parameter configs are ill-conditioned through
    the BatchNorm + ReLU (+ max-pool) stages: one ReLU whose input is within
    the forward's 1e-6 rounding difference of zero flips its mask and moves the
    gradient by ~1/sqrt(elements) of the routed tensor.  Measured
    (tools/grad_trace.py): the gradient w.r.t. the decoder-2 block output
    agrees with the oracle to 1.6e-6, the gradient w.r.t. the decoder-1 output
    (after decoder-2's ReLU routing) to 4e-3 (default_256) / 1.2e-2
    (default_clip), and every upstream gradient (ViT, patch embedding, encoder)
    inherits that.  So the whole-model bars are 3e-2 on the 28M configs, 5e-3
    on the tiny ones; the ViT backward is pinned separately, with the same
    upstream gradient on both sides, at 1e-4 (test_vit_backward_isolated)."""
    return 5e-3 if name.startswith("tiny") else 3e-2


def rel(a, b):
    a = torch.as_tensor(np.asarray(a)).double()
    b = torch.as_tensor(np.asarray(b)).double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def relnorm(a, b):
    a = torch.as_tensor(np.asarray(a)).double()
    b = torch.as_tensor(np.asarray(b)).double()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


CASES = [("tiny_64", O.TINY), ("tiny_odd", O.TINY), ("tiny_clip", O.TINY), ("default_256", {}),
         ("default_clip", {}), ("large_256", LARGE), ("tiny_cls", dict(O.TINY, use_cls_token=True))]


def build(hv, kw, precision, train):
    cfg = O.HViTConfig(**kw)
    if train:
        cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
    W = CF.weights(O.state_dict_shapes(cfg))
    m = hv.HybridViT(**cfg.as_kwargs(), precision=precision).cuda()
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    return m


@pytest.mark.parametrize("name,kw", CASES)
def test_eval_forward_fp32(hv, name, kw):
    g = golden(name)
    m = build(hv, kw, "fp32", False).eval()
    x = torch.as_tensor(g["x"]).cuda()
    with torch.no_grad():
        if "eval_attn0" in g:
            y, attn = m(x, return_attentions=True)
            for l, a in enumerate(attn):
                assert rel(a.cpu(), g[f"eval_attn{l}"]) < FP32_TOL
        else:
            y = m(x)
    torch.cuda.synchronize()
    assert tuple(y.shape) == tuple(g["eval_out"].shape)
    assert rel(y.cpu(), g["eval_out"]) < FP32_TOL, name


@pytest.mark.parametrize("name,kw", CASES)
def test_train_step_fp32(hv, name, kw):
    g = golden(name)
    m = build(hv, kw, "fp32", True).train()
    x = torch.as_tensor(g["x"]).cuda()
    y = m(x)
    loss = hv.CombinedLoss()(y, torch.as_tensor(g["target"]).cuda())
    loss.backward()
    torch.cuda.synchronize()
    assert rel(y.detach().cpu(), g["train_out"]) < FP32_TOL
    assert abs(loss.item() - float(g["train_loss"])) < 1e-4 * abs(float(g["train_loss"]))
    named = dict(m.named_parameters())
    checked = 0
    for k, p in named.items():
        gk = f"grad.{k}"
        ref_norm = float(g[f"gnorm.{k}"])
        got = p.grad.detach().cpu()
        if ref_norm > 1e-8:
            assert abs(got.double().norm().item() - ref_norm) < 5e-3 * ref_norm, k
        if gk in g:
            gr = got
            if k == "pos_encoding.pos_embed":
                gr = gr[:, : g[gk].shape[1]]
            assert relnorm(gr, g[gk]) < grad_tol(name, k), k
            checked += 1
        if f"full16.{k}" in g:  # full gradients stored as float16 (tools/gen_golden.py)
            r = g[f"full16.{k}"].astype(np.float32)
            assert relnorm(got[: r.shape[0]], r) < grad_tol(name, k), k
            checked += 1
    assert checked >= 6
    bufs = dict(m.named_buffers())
    for k in bufs:
        if f"buf.{k}" in g:
            assert rel(bufs[k].cpu(), g[f"buf.{k}"]) < 1e-4, k


@pytest.mark.parametrize("name,kw", [("tiny_64", O.TINY), ("default_256", {}), ("default_clip", {}),
                                     ("large_256", LARGE)])
def test_bf16_path(hv, name, kw):
    g = golden(name)
    m = build(hv, kw, "bf16", False).eval()
    with torch.no_grad():
        y = m(torch.as_tensor(g["x"]).cuda())
    assert rel(y.cpu(), g["eval_out"]) < BF16_TOL
    m = build(hv, kw, "bf16", True).train()
    y = m(torch.as_tensor(g["x"]).cuda())
    loss = hv.CombinedLoss()(y, torch.as_tensor(g["target"]).cuda())
    loss.backward()
    assert abs(loss.item() - float(g["train_loss"])) < 2e-2 * abs(float(g["train_loss"]))
    qk = "transformer.blocks.0.attn.qkv.weight"
    gq = dict(m.named_parameters())[qk].grad.cpu()
    assert abs(gq.double().norm().item() - float(g[f"gnorm.{qk}"])) < 0.1 * float(g[f"gnorm.{qk}"])


def test_long_clip_bf16_vs_oracle(hv):
    """A ~4 s clip: the default model on a [1, 1, 256, 496] spectrogram, 496
    tokens -- the register-resident attention's chunked N > 256 forward (8-wave
    workgroups, two 256-key chunks, online softmax) and its KMAX = 512 backward
    (data/dataset.py:297-347 pads T per batch).  bf16 eval forward
    against the fp32 CPU oracle (closed-form weights) within the bf16 bar; a
    dropout-free bf16 train step with the loss within 2 % and EVERY parameter
    gradient held to the bar of test_batch32_train_step_bf16_vs_oracle_grads:
    within 2x (+1e-2) of what torch bf16 autocast of the same oracle gives
    (one sample: the weight gradients sum over 496 rows instead of 8192, so
    their bf16 noise is larger than at B=32 -- the calibration carries that)."""
    cfg = O.HViTConfig()
    cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
    shapes = O.state_dict_shapes(cfg)
    W = CF.weights(shapes)
    x = torch.as_tensor(CF.spectrogram((1, 1, 256, 496), 81))
    t = torch.as_tensor(CF.spectrogram((1, 1, 256, 496), 82))
    m = hv.HybridViT(**cfg.as_kwargs(), precision="bf16").cuda()
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    with torch.no_grad():
        y = m.eval()(x.cuda()).cpu()
        yo = O.forward(O.make_state(shapes, W, requires_grad=False), x, cfg)
    assert m.last_num_tokens == 496
    e_fwd = rel(y, yo)
    sd = O.make_state(shapes, W, requires_grad=True)
    lo_t = O.combined_loss(O.forward(sd, x, cfg, training=True), t)
    lo_t.backward()
    lo = lo_t.item()
    sdg = {k: v.detach().cuda().requires_grad_(v.requires_grad) for k, v in sd.items()}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        yb = O.forward(sdg, x.cuda(), cfg, training=True)
    O.combined_loss(yb.float(), t.cuda()).backward()
    loss = hv.CombinedLoss()(m.train()(x.cuda()), t.cuda())
    loss.backward()
    torch.cuda.synchronize()
    worst, bad = {}, []
    for k, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), k
        got, ref, tb = p.grad.detach().cpu(), sd[k].grad, sdg[k].grad.detach().float().cpu()
        if k == "pos_encoding.pos_embed":
            got, ref, tb = got[:, :496], ref[:, :496], tb[:, :496]
        e, et = relnorm(got, ref), relnorm(tb, ref)
        grp = k.split(".")[0]
        worst[grp] = max(worst.get(grp, (0.0, 0.0, "")), (e, et, k))
        if e > 2 * et + 1e-2:
            bad.append((k, round(e, 4), round(et, 4)))
    print(f"N=496: fwd rel {e_fwd:.2e}, loss {loss.item():.6f} vs {lo:.6f}; worst rel-L2 per group (ours, autocast):",
          {g: f"{v[0]:.2e} / {v[1]:.2e} ({v[2]})" for g, v in worst.items()})
    assert e_fwd < BF16_TOL
    assert abs(loss.item() - lo) < 2e-2 * abs(lo)
    assert not bad, bad


def test_inference_fusions_match_training_graph_path(hv):
    """Inference (eval + no_grad, BASELINE config 2) takes the fused forms: eval
    BatchNorm folded into every conv block (the pooling encoder block keeping
    each 2x2 window's maximum in the conv epilogue, z never stored) and fc1
    storing gelu(h) only.  Same model, same input with grad enabled (the
    unfused eval path that keeps z and gelu'(h) for a backward): equal within
    bf16 rounding of the folded weights (each folded conv weight is rounded to
    bf16 once more than the unfused path's; measured relnorm 1.0e-2 over the
    default model's conv blocks, bar 2e-2)."""
    m = build(hv, {}, "bf16", False).eval()
    g = golden("default_256")
    x = torch.as_tensor(g["x"]).cuda()
    with torch.no_grad():
        y_fused = m(x)
    y_plain = m(x).detach()
    assert relnorm(y_fused.cpu(), y_plain.cpu()) < 2e-2
    assert rel(y_fused.cpu(), y_plain.cpu()) < 5e-2


def test_inference_reuses_prepared_weights_until_they_change(hv):
    """Repeated inference forwards reuse the packed / BN-folded conv weights
    (no weight-preparation launch after the first), bit-identical outputs; an
    in-place change of a conv weight or of a BatchNorm running statistic is
    seen by the next forward (it equals a fresh model's); a training step in
    between (train() then eval()) drops the cache."""
    import importlib

    HF = importlib.import_module("hvit_amd.functional")
    m = build(hv, {}, "bf16", False).eval()
    g = golden("default_256")
    x = torch.as_tensor(g["x"]).cuda()
    with torch.no_grad():
        y0 = m(x)
        prepared = {k: v[1] for k, v in HF._PREP.items()}
        y1 = m(x)
        assert all(HF._PREP[k][1] is t for k, t in prepared.items())  # reused, not re-prepared
        assert torch.equal(y0, y1)
        m.encoder[1].conv.weight.mul_(1.25)
        m.decoder[0].bn.running_var.mul_(2.0)
        y2 = m(x)
    fresh = build(hv, {}, "bf16", False).eval()
    fresh.load_state_dict(m.state_dict())
    with torch.no_grad():
        y3 = fresh(x)
    assert not torch.equal(y2, y1)
    assert torch.equal(y2, y3)
    m.train()
    assert not HF._PREP
    m.eval()
    with torch.no_grad():
        assert torch.equal(m(x), y2)


def test_autocast_selects_bf16(hv):
    m = build(hv, O.TINY, "auto", False).eval()
    x = torch.as_tensor(CF.spectrogram((2, 1, 64, 64), 5)).cuda()
    with torch.no_grad():
        y32 = m(x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y16 = m(x)
    assert y32.dtype == torch.float32 and y16.dtype == torch.float32
    d = (y32 - y16).abs().max().item()
    assert 0 < d < 0.05


def test_dropout_train_mode_is_seeded(hv):
    cfg = dict(O.TINY)
    m = hv.HybridViT(**cfg, precision="fp32").cuda().train()
    x = torch.as_tensor(CF.spectrogram((2, 1, 64, 64), 6)).cuda()
    torch.manual_seed(1)
    y1 = m(x)
    torch.manual_seed(1)
    y2 = m(x)
    torch.manual_seed(2)
    y3 = m(x)
    assert torch.equal(y1, y2)
    assert not torch.equal(y1, y3)
    y1.sum().backward()
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), n


def test_forward_encoder_transformer_decoder_api(hv):
    g = golden("tiny_64")
    m = build(hv, O.TINY, "fp32", False).eval()
    x = torch.as_tensor(g["x"]).cuda()
    with torch.no_grad():
        feat, skips = m.forward_encoder(x)
        for i, sk in enumerate(skips):
            assert rel(sk.cpu(), g[f"eval_enc{i}"]) < FP32_TOL
        tokens = torch.as_tensor(g["eval_tokens"]).cuda()
        f = m.forward_transformer(tokens, (feat.shape[2] // 4, feat.shape[3] // 4))
        out = m.forward_decoder(f, skips)
    assert out.shape[2:] == (16, 16)


def test_oracle_agreement_random_weights(hv):
    """Random torch-initialised weights (not the closed form), fp32, vs oracle."""
    torch.manual_seed(3)
    cfg = O.HViTConfig(**O.TINY)
    m = hv.HybridViT(**cfg.as_kwargs(), precision="fp32").eval()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.cuda()
    x = torch.rand(2, 1, 48, 80)
    with torch.no_grad():
        y = m(x.cuda()).cpu()
        yo = O.forward(sd, x, cfg)
    assert rel(y, yo) < FP32_TOL


@pytest.mark.parametrize("name,kw", [("default_256", {}), ("large_256", LARGE)])
def test_all_grads_vs_oracle(hv, name, kw):
    """Every parameter gradient of a train step (dropout off) against the CPU
    oracle's autograd on the same inputs/weights, full tensors, at grad_tol."""
    g = golden(name)
    cfg = O.HViTConfig(**kw)
    cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
    shapes = O.state_dict_shapes(cfg)
    W = CF.weights(shapes)
    x, t = torch.as_tensor(g["x"]), torch.as_tensor(g["target"])
    sd = O.make_state(shapes, W, requires_grad=True)
    O.combined_loss(O.forward(sd, x, cfg, training=True), t).backward()
    m = build(hv, kw, "fp32", True).train()
    hv.CombinedLoss()(m(x.cuda()), t.cuda()).backward()
    torch.cuda.synchronize()
    worst = {}
    for k, p in m.named_parameters():
        ref = sd[k].grad
        got = p.grad.detach().cpu()
        if k == "pos_encoding.pos_embed":
            n = 256
            assert got[:, n:].abs().max().item() == 0.0
            got, ref = got[:, :n], ref[:, :n]
        e = relnorm(got, ref)
        grp = k.split(".")[0]
        worst[grp] = max(worst.get(grp, 0.0), e)
        assert e < grad_tol(name, k), (k, e)
    print(name, {k: f"{v:.1e}" for k, v in worst.items()})


def test_batch32_eval_forward_vs_oracle(hv):
    """BASELINE config 2 batch (B=32, 256x256, default model) fp32 eval forward
    against the CPU oracle: batch-size-dependent indexing (BN partial tiles,
    split-K planning, grid limits) is exercised at the bench's M."""
    cfg = O.HViTConfig()
    shapes = O.state_dict_shapes(cfg)
    W = CF.weights(shapes)
    x = torch.as_tensor(CF.spectrogram((32, 1, 256, 256), 77))
    cap = {}
    with torch.no_grad():
        yo = O.forward(O.make_state(shapes, W), x, cfg, capture=cap)
    m = build(hv, {}, "fp32", False).eval()
    with torch.no_grad():
        y = m(x.cuda()).cpu()
    assert rel(y, yo) < FP32_TOL
    # per-sample check: no sample is corrupted while the max stays small
    per = ((y - yo).flatten(1).norm(dim=1) / yo.flatten(1).norm(dim=1))
    assert per.max().item() < 1e-4, per
    mb = build(hv, {}, "bf16", False).eval()
    with torch.no_grad():
        yb = mb(x.cuda()).cpu()
    assert rel(yb, yo) < BF16_TOL


def test_batch32_train_step_bf16_vs_oracle_grads(hv):
    """B=32 train step (BASELINE config 3 shapes, bf16, dropout off) against
    the fp32 CPU oracle: the loss, and EVERY parameter gradient per tensor
    (relative L2).  The bar is what bf16 arithmetic itself gives on this model:
    the same oracle run by torch under bf16 autocast on the GPU (its own
    rocBLAS / MIOpen kernels) is compared with the fp32 oracle the same way, and
    each of our tensors must be within 2x of that error (+1e-2): ReLU / max-pool
    routing flips and BatchNorm statistics in bf16 are inherent to the precision,
    a wrong tile, swizzle or epilogue is not."""
    cfg = O.HViTConfig()
    cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
    shapes = O.state_dict_shapes(cfg)
    W = CF.weights(shapes)
    x = torch.as_tensor(CF.spectrogram((32, 1, 256, 256), 78))
    t = torch.as_tensor(CF.spectrogram((32, 1, 256, 256), 79))
    sd = O.make_state(shapes, W, requires_grad=True)
    lo_t = O.combined_loss(O.forward(sd, x, cfg, training=True), t)
    lo_t.backward()
    lo = lo_t.item()
    # torch bf16 autocast of the same oracle (calibration of the bf16 error)
    sdg = {k: v.detach().cuda().requires_grad_(v.requires_grad) for k, v in sd.items()}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        yb = O.forward(sdg, x.cuda(), cfg, training=True)
    O.combined_loss(yb.float(), t.cuda()).backward()
    m = build(hv, {}, "bf16", True).train()
    y = m(x.cuda())
    loss = hv.CombinedLoss()(y, t.cuda())
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - lo) < 2e-2 * abs(lo)
    worst, bad = {}, []
    for k, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), k
        got, ref, tb = p.grad.detach().cpu(), sd[k].grad, sdg[k].grad.detach().float().cpu()
        if k == "pos_encoding.pos_embed":
            got, ref, tb = got[:, :256], ref[:, :256], tb[:, :256]
        e, et = relnorm(got, ref), relnorm(tb, ref)
        grp = k.split(".")[0]
        worst[grp] = max(worst.get(grp, (0.0, 0.0, "")), (e, et, k))
        if e > 2 * et + 1e-2:
            bad.append((k, round(e, 4), round(et, 4)))
    print("bf16 B=32 step, worst rel-L2 per group (ours, torch bf16 autocast):",
          {g: f"{v[0]:.2e} / {v[1]:.2e} ({v[2]})" for g, v in worst.items()})
    assert not bad, bad


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_skip_grad_handoff_matches_autograd_add(hv, precision):
    """HF.SkipGrad (a SkipFn hands its gradient to the encoder output's other
    consumer, which adds it with the bilinear backward in accumulate mode) gives
    the gradients of autograd's own add (HF.SKIPGRAD off)."""
    import sys
    HF = sys.modules["hvit_amd.functional"]
    g = golden("tiny_64")
    x, t = torch.as_tensor(g["x"]).cuda(), torch.as_tensor(g["target"]).cuda()
    grads = []
    for on in (True, False):
        HF.SKIPGRAD = on
        try:
            m = build(hv, O.TINY, precision, True).train()
            hv.CombinedLoss()(m(x), t).backward()
            grads.append({k: p.grad.detach().clone() for k, p in m.named_parameters()})
        finally:
            HF.SKIPGRAD = True
    tol = 1e-5 if precision == "fp32" else 1e-2
    for k in grads[0]:
        assert relnorm(grads[0][k].cpu(), grads[1][k].cpu()) < tol, k


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("cls", [False, True], ids=["nocls", "cls"])
def test_ln_dropout_fusion_matches_separate_passes(hv, precision, cls):
    """HF.LNDROP (the attention branch's dropout fused into LN2's backward, each
    block's MLP-branch dropout into the next consumer's LN backward through
    HF.GradHandoff) gives the gradients of the separate dropout_scale passes,
    with dropout and DropPath on (train mode, reference default rates; same
    seeds)."""
    import sys
    HF = sys.modules["hvit_amd.functional"]
    g = golden("tiny_64")
    x, t = torch.as_tensor(g["x"]).cuda(), torch.as_tensor(g["target"]).cuda()
    kw = dict(O.TINY, drop_path_rate=0.1, use_cls_token=cls)
    grads = []
    for on in (True, False):
        HF.LNDROP = on
        try:
            torch.manual_seed(5)
            m = build(hv, kw, precision, False).train()
            hv.CombinedLoss()(m(x), t).backward()
            grads.append({k: p.grad.detach().clone() for k, p in m.named_parameters()})
        finally:
            HF.LNDROP = True
    tol = 1e-5 if precision == "fp32" else 1e-2
    for k in grads[0]:
        assert relnorm(grads[0][k].cpu(), grads[1][k].cpu()) < tol, k


@pytest.mark.parametrize("kw", [{}, LARGE], ids=["default", "large"])
def test_vit_backward_isolated(hv, kw):
    """The transformer path alone (pos-embed add, every ViT block, final
    LayerNorm, to_feature_map; hybrid_vit.py:309-350, attention.py:176-300) in
    fp32 train mode with dropout off, driven by the SAME upstream gradient on
    the HIP side (forward_transformer) and the oracle side: no ReLU routing
    upstream, so every ViT / head / pos-embed gradient and the token gradient
    are pinned at 1e-4 relative L2."""
    import torch.nn.functional as F
    cfg = O.HViTConfig(**kw)
    cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
    shapes = O.state_dict_shapes(cfg)
    W = CF.weights(shapes)
    D, C, B, Hp, Wp = cfg.embed_dim, cfg.encoder_channels[-1], 2, 16, 16
    gen = torch.Generator().manual_seed(21)
    tok = torch.randn(B, Hp * Wp, D, generator=gen)
    G = torch.randn(B, C, Hp, Wp, generator=gen)
    m = build(hv, kw, "fp32", True).train()
    tk = tok.cuda().requires_grad_(True)
    out = m.forward_transformer(tk, (Hp, Wp))
    (out * G.cuda()).sum().backward()
    sd = O.make_state(shapes, W, requires_grad=True)
    to = tok.clone().requires_grad_(True)
    t = to + sd["pos_encoding.pos_embed"][:, :Hp * Wp]
    dpr = [v.item() for v in torch.linspace(0, cfg.drop_path_rate, cfg.num_layers)]
    for l in range(cfg.num_layers):
        t, _ = O.vit_block(sd, f"transformer.blocks.{l}", t, cfg, dpr[l], True)
    t = F.layer_norm(t, (D,), sd["transformer.norm.weight"], sd["transformer.norm.bias"], 1e-5)
    f = F.linear(t, sd["to_feature_map.weight"], sd["to_feature_map.bias"])
    ref = f.transpose(1, 2).reshape(B, C, Hp, Wp)
    (ref * G).sum().backward()
    assert rel(out.detach().cpu(), ref.detach()) < 1e-5
    assert relnorm(tk.grad.cpu(), to.grad) < 1e-4
    n = 0
    for k, p in m.named_parameters():
        if not (k.startswith("transformer") or k.startswith("to_feature_map") or k.startswith("pos_encoding")):
            continue
        r = sd[k].grad
        got = p.grad.detach().cpu()
        if k == "pos_encoding.pos_embed":
            got, r = got[:, :Hp * Wp], r[:, :Hp * Wp]
        assert relnorm(got, r) < 1e-4, k
        n += 1
    assert n == 12 * cfg.num_layers + 5


def _f8(x):
    """round to OCP e4m3 (float8_e4m3fn) and back"""
    return x.to(torch.float8_e4m3fn).to(x.dtype)


def _pow2(amax):
    """the fp8 kernel's power-of-two scale 2^floor(log2(448 / amax))"""
    amax = amax.detach().float()
    r = torch.where(amax > 0, 448.0 / amax.clamp_min(1e-30), torch.ones_like(amax))
    return torch.exp2(torch.floor(torch.log2(r)))


def _mhsa_fp8_emulated(sd, pfx, x, H, p_attn, p, training, want_attn=False):
    """O.mhsa with the fp8 attention forward's roundings (attention_fp8.hip:
    per-(b,h) K / V and per-query Q power-of-two scales, e4m3 q, k, v and
    256 exp(s - max), normaliser from the unrounded sum) as straight-through
    values: the backward sees the unrounded operands, as the bf16 backward of
    the fp8 path does.  Dropout off (the test's configuration)."""
    import torch.nn.functional as F
    B, N, C = x.shape
    hd = C // H
    qkv = F.linear(x, sd[f"{pfx}.qkv.weight"], sd[f"{pfx}.qkv.bias"])
    qkv = qkv.reshape(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    st = lambda t, r: t + (r - t).detach()  # noqa: E731
    sq = _pow2(q.abs().amax(dim=3, keepdim=True)).to(q.dtype)
    sk = _pow2(k.abs().amax(dim=(2, 3), keepdim=True)).to(k.dtype)
    sv = _pow2(v.abs().amax(dim=(2, 3), keepdim=True)).to(v.dtype)
    q8, k8, v8 = st(q, _f8(q * sq) / sq), st(k, _f8(k * sk) / sk), st(v, _f8(v * sv) / sv)
    s = (q8 @ k8.transpose(-2, -1)).float() * (hd ** -0.5)
    u = torch.exp(s - s.amax(-1, keepdim=True).detach())
    o = (st(u, _f8(u * 256.0) / 256.0) @ v8.float()) / u.sum(-1, keepdim=True)
    o = o.to(x.dtype).transpose(1, 2).reshape(B, N, C)
    o = F.linear(o, sd[f"{pfx}.proj.weight"], sd[f"{pfx}.proj.bias"])
    return o, None


def _config5_step_grads(hv, monkeypatch, B, sx, stg, record):
    import json
    cfg = O.HViTConfig(**LARGE)
    cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
    shapes = O.state_dict_shapes(cfg)
    W = CF.weights(shapes)
    x = torch.as_tensor(CF.spectrogram((B, 1, 256, 256), sx))
    t = torch.as_tensor(CF.spectrogram((B, 1, 256, 256), stg))
    sd = O.make_state(shapes, W, requires_grad=True)
    lo_t = O.combined_loss(O.forward(sd, x, cfg, training=True), t)
    lo_t.backward()
    lo = lo_t.item()
    tgrads = {}
    for name in ("bf16", "fp8"):
        sdg = {k: v.detach().cuda().requires_grad_(v.requires_grad) for k, v in sd.items()}
        with monkeypatch.context() as mp:
            if name == "fp8":
                mp.setattr(O, "mhsa", _mhsa_fp8_emulated)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                yb = O.forward(sdg, x.cuda(), cfg, training=True)
            O.combined_loss(yb.float(), t.cuda()).backward()
        tgrads[name] = {k: v.grad.detach().float().cpu() for k, v in sdg.items() if v.grad is not None}
    table, bad = {}, []
    for name in ("bf16", "fp8"):
        m = hv.HybridViT(**cfg.as_kwargs(), precision="bf16",
                        attention_precision="fp8" if name == "fp8" else None).cuda().train()
        m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
        loss = hv.CombinedLoss()(m(x.cuda()), t.cuda())
        loss.backward()
        torch.cuda.synchronize()
        assert abs(loss.item() - lo) < 2e-2 * abs(lo), (name, loss.item(), lo)
        for k, p in m.named_parameters():
            assert p.grad is not None and torch.isfinite(p.grad).all(), (name, k)
            got, ref, tb = p.grad.detach().cpu(), sd[k].grad, tgrads[name][k]
            if k == "pos_encoding.pos_embed":
                got, ref, tb = got[:, :256], ref[:, :256], tb[:, :256]
            e, et = relnorm(got, ref), relnorm(tb, ref)
            grp = k.split(".")[0] if not k.startswith("transformer.blocks") else "transformer." + k.split(".")[3]
            cur = table.setdefault(name, {}).get(grp)
            if cur is None or e > cur[0]:
                table[name][grp] = (e, et, k)
            if e > 2 * et + 1e-2:
                bad.append((name, k, round(e, 4), round(et, 4)))
    out = {n: {g: {"ours": v[0], "torch_emulation": v[1], "worst_tensor": v[2]} for g, v in d.items()}
           for n, d in table.items()}
    print(f"config 5 B={B} step, worst rel-L2 per group:", json.dumps(out, indent=1))
    if os.environ.get("HVIT_RECORD"):
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", record), "w") as f:
            json.dump({"batch": B, "loss_oracle": lo, "groups": out, "violations": bad}, f, indent=1)
    assert not bad, bad


def test_large_config_fp8_train_step_grads(hv, monkeypatch):
    """BASELINE config 5 train step (D=768 / 12 heads / 12 layers, bf16, dropout
    off, B=4) with the fp8 attention forward: the loss and EVERY parameter
    gradient per tensor (relative L2) against the fp32 CPU oracle.  Bars
    calibrated as the bf16 B=32 test's: torch bf16 autocast of the oracle gives
    the bf16 error e_tb, and the same with the attention core replaced by an
    emulation of the fp8 forward's roundings (straight-through, bf16 backward)
    gives the fp8 error e_t8; our bf16 path must stay within 2 e_tb + 1e-2 and
    our fp8 path within 2 e_t8 + 1e-2 per tensor.  The per-group table goes to
    gpurun_out/fp8_grad_calibration.json when HVIT_RECORD is set."""
    _config5_step_grads(hv, monkeypatch, 4, 80, 81, "fp8_grad_calibration.json")


def test_large_config_b16_train_step_grads(hv, monkeypatch):
    """BASELINE config 5 at its own batch, B=16 (M = 4,096 token rows: the
    bench's tile counts, split-K plans and LayerNorm row paths), bf16 and fp8
    attention: the loss and every parameter gradient per tensor against the
    fp32 CPU oracle, bars calibrated as in the B=4 test (2x torch bf16 autocast
    of the oracle, with the fp8 forward's roundings emulated for the fp8 path,
    + 1e-2).  Table: gpurun_out/fp8_grad_calibration_b16.json (HVIT_RECORD)."""
    _config5_step_grads(hv, monkeypatch, 16, 82, 83, "fp8_grad_calibration_b16.json")


def test_large_config_fp8_attention(hv):
    """BASELINE config 5: the D=768 / 12-head / 12-layer model in bf16 with the
    fp8 attention forward, against the reference's fp32 golden output at the
    bf16 bar, and one train step (bf16 attention backward) with the loss at the
    bf16 bar and finite gradients."""
    g = golden("large_256")
    cfg = O.HViTConfig(**LARGE)
    W = CF.weights(O.state_dict_shapes(cfg))
    m = hv.HybridViT(**cfg.as_kwargs(), precision="bf16", attention_precision="fp8").cuda().eval()
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    with torch.no_grad():
        y = m(torch.as_tensor(g["x"]).cuda())
    assert rel(y.cpu(), g["eval_out"]) < BF16_TOL
    cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
    m = hv.HybridViT(**cfg.as_kwargs(), precision="bf16", attention_precision="fp8").cuda().train()
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    loss = hv.CombinedLoss()(m(torch.as_tensor(g["x"]).cuda()), torch.as_tensor(g["target"]).cuda())
    loss.backward()
    assert abs(loss.item() - float(g["train_loss"])) < 2e-2 * abs(float(g["train_loss"]))
    for k, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), k
