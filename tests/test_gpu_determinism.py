"""GPU: the train step is deterministic and reads no memory it did not write.

Every reduction on the step is a fixed-order sum of per-workgroup partial rows
(no float atomics: GEMM bias column sums, BatchNorm backward sums, the fused
first block's sums, LayerNorm dgamma / dbeta, the qkv bias rows of the
attention backward, hvit_reduce_rows), so

* a kernel's outputs, workspaces and partial-row buffers pre-filled with NaN
  give the same bits as the same buffers pre-filled with zeros (no read of an
  unwritten element: a pad lane of a partial tile, an LDS region read before it
  is written, a workspace row no workgroup covers), and
* a whole forward + CombinedLoss + backward repeated from the same parameters
  and dropout seed gives bit-identical loss and gradients, also when the
  allocator's cached blocks were poisoned with NaN in between.
"""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib(hv):
    return hv._lib


def _s():
    return torch.cuda.current_stream().cuda_stream


def _fill(ts, v):
    for t in ts:
        if t.dtype.is_floating_point:
            t.fill_(v)
        else:
            t.fill_(-1 if v != v else 0)  # integer buffers: all bits set vs zero


@pytest.mark.parametrize("B,N,H,hd,p", [(8, 256, 8, 64, 0.1), (4, 240, 8, 64, 0.1), (2, 300, 2, 64, 0.1),
                                        (2, 260, 4, 16, 0.1), (3, 100, 2, 64, 0.0)])
def test_attention_poisoned_buffers_bitwise(hv, B, N, H, hd, p):
    """One forward (keep bits) + one backward (fused qkv bias rows) with every
    output / workspace / partial-row buffer NaN-filled vs zero-filled: equal bit
    for bit (the first-call record of round 3)."""
    l = _lib(hv)
    D = H * hd
    torch.manual_seed(3)
    qkv = (torch.randn(B * N, 3 * D, device=DEV) * 0.7).to(torch.bfloat16)
    go = torch.randn(B * N, D, device=DEV).to(torch.bfloat16)
    dr = l.dropout(p, 17, 77) if p > 0 else None
    rows = l.lib().hvit_mhsa_bias_rows(l.BF16, B, N, H, hd)
    nkb = l.lib().hvit_mhsa_keep_bits_elems(B, N, H)
    outs = []
    for v in (float("nan"), 0.0):
        o = torch.empty(B * N, D, device=DEV, dtype=torch.bfloat16)
        lse = torch.empty(B, H, N, device=DEV)
        kb = torch.empty(nkb, dtype=torch.int32, device=DEV)
        dqkv = torch.empty_like(qkv)
        delta = torch.empty(B, H, N, device=DEV)
        parts = torch.empty(rows, 3 * D, device=DEV)
        _fill((o, lse, kb, dqkv, delta, parts), v)
        l.call("hvit_mhsa_fwd_kb", l.BF16, qkv.data_ptr(), B, N, H, hd, hd ** -0.5, dr, o.data_ptr(), lse.data_ptr(),
               kb.data_ptr(), _s())
        l.call("hvit_mhsa_bwd_db", l.BF16, qkv.data_ptr(), o.data_ptr(), go.data_ptr(), lse.data_ptr(), B, N, H, hd,
               hd ** -0.5, dr, kb.data_ptr(), dqkv.data_ptr(), delta.data_ptr(), parts.data_ptr(), _s())
        outs.append((o, lse, dqkv, parts))
    torch.cuda.synchronize()
    for a, b, name in zip(outs[0], outs[1], ("o", "lse", "dqkv", "bias_rows")):
        assert torch.isfinite(a.float()).all(), name
        assert torch.equal(a, b), name


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("M,N", [(1024, 512), (32, 131072), (131072, 64), (8192, 1536), (5, 12), (0, 64)])
def test_reduce_rows_deterministic(hv, dt, M, N):
    """hvit_reduce_rows: fixed summation order (repeat calls bit-identical, the
    accumulate form adds onto the destination), f64 reference within f32
    rounding; M = 0 writes zeros."""
    l = _lib(hv)
    tdt = torch.float32 if dt == "f32" else torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(M + N)
    x = torch.randn(max(M, 1), N, device=DEV, generator=g).to(tdt)
    code = l.F32 if dt == "f32" else l.BF16
    res = []
    for _ in range(3):
        out = torch.full((N,), float("nan"), device=DEV)
        l.call("hvit_reduce_rows", x.data_ptr(), code, M, N, N, 0, out.data_ptr(), _s())
        res.append(out)
    acc = torch.ones(N, device=DEV)
    l.call("hvit_reduce_rows", x.data_ptr(), code, M, N, N, 1, acc.data_ptr(), _s())
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1]) and torch.equal(res[0], res[2])
    want = x[:M].double().sum(0) if M > 0 else torch.zeros(N, device=DEV, dtype=torch.float64)
    bar = x[:M].double().abs().sum(0) * 2e-6 + 1e-6 if M > 0 else torch.full((N,), 1e-30, device=DEV)
    assert ((res[0].double() - want).abs() <= bar).all()
    assert torch.equal(acc, res[0] + 1.0) or ((acc.double() - want - 1.0).abs() <= bar + 1e-6).all()


KW = dict(encoder_channels=[8, 16, 32], embed_dim=64, num_heads=4, num_layers=2, decoder_channels=[32, 16, 8, 1])


def _poison_cache(value):
    """Fill the caching allocator's free blocks with ``value``: large-pool
    blocks by one big allocation, small-pool blocks (< 1 MB requests) by many
    small ones, freed again so the next step's allocations reuse them."""
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    big = torch.empty(256 << 20, dtype=torch.uint8, device=DEV)
    big.view(torch.float32).fill_(value)
    small = [torch.empty(256 << 10, dtype=torch.uint8, device=DEV) for _ in range(256)]
    for t in small:
        t.view(torch.float32).fill_(value)
    torch.cuda.synchronize()
    del big, small


@pytest.mark.parametrize("kw", [dict(KW, precision="bf16"), dict(KW, embed_dim=128, num_heads=2, precision="bf16"),
                                dict(precision="bf16")], ids=["hd16", "hd64", "default"])
def test_train_step_bitwise_repeatable_poisoned_cache(hv, kw):
    """forward + CombinedLoss + backward (dropout 0.1 everywhere, DropPath,
    train-mode BatchNorm) run three times from the same parameters and dropout
    state -- on a zero-filled allocator cache, a NaN-poisoned one and a zero
    one again: loss, every gradient and every BatchNorm running statistic are
    bit-identical."""
    torch.manual_seed(0)
    m0 = hv.HybridViT(**kw).to(DEV).train()
    crit = hv.CombinedLoss()
    shape = (2, 1, 48, 64) if "embed_dim" in kw else (4, 1, 256, 256)
    g = torch.Generator().manual_seed(8)
    x = torch.rand(shape, generator=g).to(DEV)
    t = torch.rand(shape, generator=g).to(DEV)
    runs = []
    for fill in (0.0, float("nan"), 0.0):
        m = copy.deepcopy(m0)
        m.set_dropout_state(4242)
        _poison_cache(fill)
        loss = crit(m(x), t)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters()},
                     {n: b.clone() for n, b in m.named_buffers()}))
    for r in runs[1:]:
        assert torch.equal(runs[0][0], r[0])
        for n in runs[0][1]:
            assert torch.isfinite(r[1][n]).all(), n
            assert torch.equal(runs[0][1][n], r[1][n]), n
        for n in runs[0][2]:
            assert torch.equal(runs[0][2][n], r[2][n]), n


@pytest.mark.parametrize("kw", [dict(KW, embed_dim=128, num_heads=2, precision="bf16"), dict(precision="bf16")],
                         ids=["hd64", "default"])
def test_side_stream_weight_gradients_equal_single_stream(hv, kw):
    """Weight gradients issued on the side stream (functional.SIDE, joined back
    by the autograd final callback) equal the single-stream backward bit for
    bit, and a second backward that accumulates (its launches stay on the
    backward's stream) adds to them correctly."""
    import sys

    HF = sys.modules["hvit_amd.functional"]
    torch.manual_seed(0)
    m0 = hv.HybridViT(**kw).to(DEV).train()
    crit = hv.CombinedLoss()
    shape = (2, 1, 48, 64) if "embed_dim" in kw else (4, 1, 256, 256)
    g = torch.Generator().manual_seed(9)
    x = torch.rand(shape, generator=g).to(DEV)
    t = torch.rand(shape, generator=g).to(DEV)
    runs = []
    old, oldg = HF.SIDE, HF.WGRAD_GROUP
    HF.WGRAD_GROUP = False  # (the per-Linear weight gradients on either stream; the grouped launch is not)
    try:
        for side in (False, True):
            HF.SIDE = side
            m = copy.deepcopy(m0)
            m.set_dropout_state(77)
            crit(m(x), t).backward()
            first = {n: p.grad.clone() for n, p in m.named_parameters()}
            crit(m(x), t).backward()  # accumulates (.grad exists): the single-stream form
            torch.cuda.synchronize()
            runs.append((first, {n: p.grad.clone() for n, p in m.named_parameters()}))
    finally:
        HF.SIDE, HF.WGRAD_GROUP = old, oldg
    for n in runs[0][0]:
        assert torch.equal(runs[0][0][n], runs[1][0][n]), n
        assert torch.equal(runs[0][1][n], runs[1][1][n]), n
