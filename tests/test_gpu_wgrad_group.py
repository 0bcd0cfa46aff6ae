"""GPU: the grouped weight-gradient launch (hvit_linear_wgrad_group, round 6).

dW_p[n, k] = dy_p[:, :n]^T x_p[:, :k] for several ViT Linears at once
(attention.py:55,58 qkv / proj, components.py:224,227 fc1 / fc2).  The
reference is torch fp32 arithmetic on the same bf16 operands, so the only
legitimate difference is f32 accumulation order (bar ACC * max|ref|,
element-wise, as tests/test_gpu_bf16_exact.py).  Cases cover every plan
shape: whole-tile rounds plus split remainder tiles (6 blocks at B = 32: 288
tiles on 256 CUs), remainder tiles only (2 blocks), several whole rounds
(config 5: 12 blocks, D = 768, B = 16), a single problem split into many
pieces, and strided dy (the qkv slice of a wider buffer).  Results must be
bit-identical from run to run (fixed-order sums), and the model's parameter
gradients equal the per-Linear path's within the same bar."""

import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16
ACC = 2e-5


def vit_problems(layers, M, D, hid, seed=0, wide=False):
    g = torch.Generator(device=DEV).manual_seed(seed)
    probs = []
    for _ in range(layers):
        for n, k in ((D, hid), (hid, D), (D, D), (3 * D, D)):
            ldy = n + 256 if wide else n  # a wider buffer: dy is a column slice
            dy = (torch.randn(M, ldy, device=DEV, generator=g) * 0.5).to(BF)[:, :n]
            x = (torch.randn(M, k, device=DEV, generator=g) * 0.5).to(BF)
            probs.append((dy, x, n, k))
    return probs


def run_group(hv, probs, M):
    L = hv._lib
    arr = (L.WgradProb * len(probs))()
    outs = []
    for i, (dy, x, n, k) in enumerate(probs):
        dw = torch.full((n, k), float("nan"), device=DEV)
        outs.append(dw)
        arr[i] = L.WgradProb(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), dw.data_ptr(), n, k)
    ws = torch.empty(int(L.lib().hvit_linear_wgrad_group_ws()), device=DEV)
    tk = torch.zeros(int(L.lib().hvit_linear_wgrad_group_tickets()), dtype=torch.int32, device=DEV)
    L.call("hvit_linear_wgrad_group", L.BF16, M, arr, len(probs), ws.data_ptr(), ws.numel(), tk.data_ptr(),
           tk.numel(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(tk.abs().sum()) == 0, "ticket counters must be left zeroed"
    return outs


def check(outs, probs):
    for i, ((dy, x, n, k), dw) in enumerate(zip(probs, outs)):
        ref = (dy.float().t() @ x.float()).double()
        d = (dw.double() - ref).abs()
        bound = ACC * ref.abs().max().item()
        bad = int((d > bound).sum()) + int(torch.isnan(dw).sum())
        assert bad == 0, f"problem {i} ({n}x{k}): {bad} elements off (max |d| {d.max().item():.3e}, bound {bound:.3e})"


@pytest.fixture(params=[6, 2, 0], ids=["ring32x4w16", "ring32x4", "ring64x2"])
def cfg(request, hv):
    """Tile configurations (hvit_gemm_tune(7, v)): the default 32-deep four-stage ring on 16 waves, on 8, and the
    64-deep two-stage ring of gemm_ring.h."""
    old = hv._lib.lib().hvit_gemm_tune(7, request.param)
    yield request.param
    hv._lib.lib().hvit_gemm_tune(7, old)


@pytest.mark.parametrize("layers,M,D,hid", [
    (6, 8192, 512, 2048),   # B=32 default model: 288 tiles -> 1 round + 32 tiles in 8 pieces
    (2, 8192, 512, 2048),   # 96 tiles: remainder pieces only
    (12, 4096, 768, 3072),  # config 5 (B=16): 1296 tiles -> 5 rounds + 16 tiles in 16 pieces
    (1, 1024, 512, 2048),   # 48 tiles, short token range
])
def test_wgrad_group_matches_fp32(hv, cfg, layers, M, D, hid):
    torch.backends.cuda.matmul.allow_tf32 = False
    probs = vit_problems(layers, M, D, hid)
    check(run_group(hv, probs, M), probs)


def test_wgrad_group_single_problem_many_pieces_and_strided_dy(hv, cfg):
    probs = vit_problems(1, 8192, 512, 2048, seed=3, wide=True)[2:3]  # proj: 4 tiles, 64 pieces each
    check(run_group(hv, probs, 8192), probs)
    probs = vit_problems(1, 8192, 512, 2048, seed=4, wide=True)
    check(run_group(hv, probs, 8192), probs)


@pytest.mark.parametrize("B,H,C,P", [(32, 64, 256, 4), (4, 64, 256, 4), (2, 32, 64, 4), (4, 32, 128, 2)])
def test_wgrad_group_patch_embedding(hv, B, H, C, P):
    """A patch-embedding weight gradient (Conv2d k = stride = P on an NHWC map) in
    the same launch as ViT problems: packed [co][ky][kx][c] result vs torch fp32
    on the explicitly gathered patches (components.py:275-280)."""
    L = hv._lib
    g = torch.Generator(device=DEV).manual_seed(11)
    D = 512
    Hp = H // P
    M = B * Hp * Hp
    feat = (torch.randn(B, H, H, C, device=DEV, generator=g) * 0.5).to(BF)
    gd = (torch.randn(M, D, device=DEV, generator=g) * 0.5).to(BF)
    assert L.lib().hvit_linear_wgrad_group_patch_ok(L.BF16, M, D, P, H, H, C) == 1
    patches = feat.view(B, Hp, P, Hp, P, C).permute(0, 1, 3, 2, 4, 5).reshape(M, P * P * C)
    ref = (gd.float().t() @ patches.float()).double()
    vit = vit_problems(1, M, 512, 2048, seed=12)
    arr = (L.WgradProb * (len(vit) + 1))()
    outs = []
    for i, (dy, x, n, k) in enumerate(vit):
        dw = torch.full((n, k), float("nan"), device=DEV)
        outs.append(dw)
        arr[i] = L.WgradProb(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), dw.data_ptr(), n, k)
    dwp = torch.full((D, P * P * C), float("nan"), device=DEV)
    arr[len(vit)] = L.WgradProb(gd.data_ptr(), D, feat.data_ptr(), 0, dwp.data_ptr(), D, P * P * C, P, H, H, C)
    ws = torch.empty(int(L.lib().hvit_linear_wgrad_group_ws()), device=DEV)
    tk = torch.zeros(int(L.lib().hvit_linear_wgrad_group_tickets()), dtype=torch.int32, device=DEV)
    L.call("hvit_linear_wgrad_group", L.BF16, M, arr, len(vit) + 1, ws.data_ptr(), ws.numel(), tk.data_ptr(),
           tk.numel(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    check(outs, vit)
    d = (dwp.double() - ref).abs()
    bound = ACC * ref.abs().max().item()
    bad = int((d > bound).sum()) + int(torch.isnan(dwp).sum())
    assert bad == 0, f"patch dW: {bad} elements off (max |d| {d.max().item():.3e}, bound {bound:.3e})"


def test_wgrad_group_deterministic(hv, cfg):
    probs = vit_problems(6, 8192, 512, 2048, seed=5)
    a = run_group(hv, probs, 8192)
    b = run_group(hv, probs, 8192)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def test_wgrad_group_rejects_bad_shapes(hv):
    L = hv._lib
    assert L.lib().hvit_linear_wgrad_group_ok(L.BF16, 8192, 512, 2048) == 1
    assert L.lib().hvit_linear_wgrad_group_ok(L.BF16, 8200, 512, 2048) == 0  # tokens % 64
    assert L.lib().hvit_linear_wgrad_group_ok(L.BF16, 8192, 320, 512) == 0   # n_out % 256
    assert L.lib().hvit_linear_wgrad_group_ok(L.F32, 8192, 512, 512) == 0
    dy = torch.zeros(8192, 320, dtype=BF, device=DEV)
    with pytest.raises(RuntimeError, match="wgrad_group"):
        run_group(hv, [(dy, dy, 320, 320)], 8192)


def test_model_grads_grouped_equal_per_linear(hv):
    """The bf16 train step's ViT weight gradients with the grouped launch equal
    the per-Linear split-K path's within the accumulation-order bar; every other
    gradient within f32 summation-order noise (the data-gradient chain is the
    same launches)."""
    HF = sys.modules["hvit_amd.functional"]
    torch.manual_seed(0)
    m = hv.HybridViT(dropout=0.0, attn_dropout=0.0, drop_path_rate=0.0, precision="bf16").cuda().train()
    x = torch.rand(8, 1, 256, 256, device=DEV)
    t = torch.rand(8, 1, 256, 256, device=DEV)
    loss_fn = hv.CombinedLoss()
    grads = {}
    for mode in (False, True):
        HF.WGRAD_GROUP = mode
        try:
            m.zero_grad(set_to_none=True)
            loss_fn(m(x), t).backward()
            torch.cuda.synchronize()
            grads[mode] = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
        finally:
            HF.WGRAD_GROUP = True
    assert not HF._WG_QUEUE, "the backward's final callback must flush the queue"
    assert HF.WG_FIXUPS == 0, "autograd must adopt the queued gradients (no copy of an unwritten tensor)"
    assert not any(HF._SIDE_PENDING.values()), "pending side jobs must be carried or flushed"
    assert not any(HF._WG_AFTER.values()), "launches deferred to the flush must have run"
    for n, g0 in grads[False].items():
        g1 = grads[True][n]
        if n == "patch_embed.projection.weight" or (
                n.startswith("transformer.blocks.") and n.endswith(("attn.qkv.weight", "attn.proj.weight",
                                                                    "mlp.net.0.weight", "mlp.net.3.weight"))):
            bound = 1e-4 * g0.abs().max().item() + 1e-12
            assert (g1 - g0).abs().max().item() <= bound, n
        else:
            # the data-gradient chain is the same; the LayerNorm / bias partial-row sums the grouped mode
            # defers to a later launch add the same rows in another fixed order (a wave per granule)
            bound = 1e-5 * g0.abs().max().item() + 1e-12
            assert (g1 - g0).abs().max().item() <= bound, n
