"""GPU: the fused first encoder block (csrc/c1block.hip, functional.C1BlockFn)
against a plain PyTorch fp32 reference of the same module chain
(ConvBlock components.py:55-85 with Cin = 1: conv3x3 no bias -> BatchNorm2d
(train: batch statistics + running-stat update; eval: running statistics) ->
ReLU -> Dropout2d -> MaxPool2d) and against the unfused library path
(hvit_conv_fwd + hvit_bn_act_* + hvit_conv_wgrad, ConvBNActFn).

Operands are rounded to the compute dtype before the reference sees them, so
the f32 path is held to f32 accumulation-order error and the bf16 path to the
rounding of its bf16 output (z itself stays f32 inside the fused kernels).
Dropout2d masks are the numpy mirror of the counter hash (conftest.keep_mask)."""

import sys

import pytest
import torch
import torch.nn.functional as F

from conftest import keep_mask

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def HF(hv):
    torch.backends.cudnn.allow_tf32 = False
    return sys.modules["hvit_amd.functional"]


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def reference(x, w, gamma, beta, rm, rv, training, p, seed, site, pool, momentum=0.1, eps=1e-5):
    """torch fp32 ConvBlock (NCHW); returns y and updates rm / rv in place."""
    N = x.shape[0]
    C = w.shape[0]
    z = F.conv2d(x, w, None, 1, 1)
    bn = F.batch_norm(z, rm, rv, gamma, beta, training, momentum, eps)
    y = F.relu(bn)
    if training and p > 0:
        m = torch.as_tensor(keep_mask(seed, site, N * C, p).reshape(N, C), device=DEV).float() / (1 - p)
        y = y * m[:, :, None, None]
    return F.max_pool2d(y, pool) if pool > 1 else y


CASES = [
    # N, H, W, C, pool, p
    (2, 32, 32, 64, 2, 0.0),
    (3, 15, 17, 16, 2, 0.3),   # odd edges: pixels outside every pooling window
    (2, 16, 24, 128, 1, 0.1),
    (1, 9, 8, 8, 2, 0.5),
    (2, 64, 251, 64, 2, 0.1),  # the model's 2 s clip width
    (2, 40, 36, 32, 2, 0.2),
]


@pytest.fixture
def impl(HF, request):
    """knob 1: the bf16 matrix-core kernels where they apply; 0: VALU kernels."""
    old = HF.L.lib().hvit_gemm_tune(1, request.param)
    yield request.param
    HF.L.lib().hvit_gemm_tune(1, old)


@pytest.mark.parametrize("dt,impl", [("f32", 1), ("bf16", 1), ("bf16", 0)], indirect=["impl"])
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("training", [True, False])
def test_c1block_matches_torch(HF, dt, impl, case, training):
    L = HF.L
    N, H, W, C, pool, p = case
    tdt = torch.float32 if dt == "f32" else torch.bfloat16
    dtc = L.F32 if dt == "f32" else L.BF16
    torch.manual_seed(N * 100 + C + W)
    x = torch.randn(N, 1, H, W, device=DEV).to(tdt).float()
    w = (torch.randn(C, 1, 3, 3, device=DEV) / 3).to(tdt).float()
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.3
    rm0, rv0 = torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5
    seed, site = 1234, 100
    # reference
    xr = x.clone()
    wr, gr, br = (t.clone().requires_grad_(True) for t in (w, gamma, beta))
    rm_r, rv_r = rm0.clone(), rv0.clone()
    yr = reference(xr, wr, gr, br, rm_r, rv_r, training, p, seed, site, pool)
    gy = torch.randn_like(yr).to(tdt).float()
    yr.backward(gy)
    # fused library path
    xa = x.permute(0, 2, 3, 1).contiguous().to(tdt)
    wa, ga, ba = (t.clone().requires_grad_(True) for t in (w, gamma, beta))
    rm_a, rv_a = rm0.clone(), rv0.clone()
    nbt = torch.zeros((), dtype=torch.long, device=DEV)
    assert HF.c1block_ok(xa, None, wa, 1, pool)
    y = HF.C1BlockFn.apply(xa, wa, ga, ba, rm_a, rv_a, nbt, pool, training, HF.Drop(p, seed, site), 0.1, 1e-5,
                           dtc)
    y.backward(gy.permute(0, 2, 3, 1).contiguous().to(tdt))
    yn = y.float().permute(0, 3, 1, 2)
    if dt == "f32":
        assert rel(yn, yr) < 1e-5
    else:  # one bf16 rounding of an f32 value (either neighbour)
        bound = yr.abs() * 2.0 ** -7 + 1e-5 * yr.abs().max()  # z and the statistics differ in summation order
        assert int(((yn - yr).abs() > bound).sum()) == 0
    tol = 1e-4
    assert rel(wa.grad, wr.grad) < tol
    if training:
        assert rel(ga.grad, gr.grad) < tol
        assert rel(ba.grad, br.grad) < tol
        assert rel(rm_a, rm_r) < 1e-5 and rel(rv_a, rv_r) < 1e-5
        assert int(nbt) == 1
    else:
        assert rel(ga.grad, gr.grad) < tol and rel(ba.grad, br.grad) < tol
        assert torch.equal(rm_a, rm0) and torch.equal(rv_a, rv0)


@pytest.mark.parametrize("training", [True, False])
def test_c1block_matches_unfused_path(HF, training):
    """Fused and unfused library paths on the model's enc0 shape class, both
    against the torch fp32 reference: the fused one (z and dz never rounded to
    bf16) is at least as accurate.  Eval mode included: both paths give the
    BatchNorm parameters their gradient."""
    L = HF.L
    N, H, W, C, pool, p = 4, 256, 256, 64, 2, 0.1
    torch.manual_seed(7)
    xa = torch.randn(N, H, W, 1, device=DEV).to(torch.bfloat16)
    w = (torch.randn(C, 1, 3, 3, device=DEV) / 3).to(torch.bfloat16).float()
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.3
    gy = torch.randn(N, H // 2, W // 2, C, device=DEV).to(torch.bfloat16)
    seed, site = 55, 100
    wr, gr, br = (t.clone().requires_grad_(True) for t in (w, gamma, beta))
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    yr = reference(xa.float().permute(0, 3, 1, 2), wr, gr, br, rm, rv, training, p, seed, site, pool)
    yr.backward(gy.float().permute(0, 3, 1, 2))
    ref = (yr.detach().permute(0, 2, 3, 1), wr.grad, gr.grad, br.grad, rm, rv)
    errs = {}
    for fused in (True, False):
        wa, ga, ba = (t.clone().requires_grad_(True) for t in (w, gamma, beta))
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        nbt = torch.zeros((), dtype=torch.long, device=DEV)
        d = HF.Drop(p, seed, site)
        if fused:
            y = HF.C1BlockFn.apply(xa, wa, ga, ba, rm, rv, nbt, pool, training, d, 0.1, 1e-5, L.BF16)
        else:
            y = HF.ConvBNActFn.apply(xa, None, wa, ga, ba, rm, rv, nbt, 1, pool, training, d, 0.1, 1e-5, L.BF16)
        y.backward(gy)
        got = (y.float(), wa.grad, ga.grad, ba.grad, rm, rv)
        errs[fused] = [rel(a, b) for a, b in zip(got, ref)]
    fe, ue = errs[True], errs[False]
    assert fe[0] < 1e-2 and max(fe[1:4]) < 1e-3 and max(fe[4:]) < 1e-5, fe
    assert max(ue[1:4]) < 1e-1, ue  # the unfused path rounds z and dz to bf16 in HBM
    for i in range(1, 4):
        assert fe[i] <= ue[i] * 1.5 + 1e-6, (i, fe, ue)


def test_c1block_graph_seed_word(HF):
    """The Dropout2d mask follows the device seed word (seed ^ *seed_ptr)."""
    L = HF.L
    N, H, W, C = 2, 16, 16, 32
    x = torch.randn(N, H, W, 1, device=DEV)
    w = torch.randn(C, 1, 3, 3, device=DEV)
    gamma, beta = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    word = torch.tensor([0x5151], dtype=torch.int64, device=DEV)
    ys = []
    for seed, t in ((0x5151 ^ 77, None), (77, word)):
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        nbt = torch.zeros((), dtype=torch.long, device=DEV)
        ys.append(HF.C1BlockFn.apply(x, w, gamma, beta, rm, rv, nbt, 1, True, HF.Drop(0.5, seed, 100, t), 0.1,
                                     1e-5, L.F32))
    assert torch.equal(ys[0], ys[1])


def test_c1block_rejects_bad_geometry(HF):
    L = HF.L
    x = torch.randn(1, 8, 8, 2, device=DEV)
    g = HF.geom(x, 2, None, 0, 1, 8, 8, 1, 3, 1, 1, 16)
    m = torch.zeros(16, device=DEV)
    y = torch.empty(1, 4, 4, 16, device=DEV)
    with pytest.raises(RuntimeError, match="Cin = 1"):
        L.call("hvit_c1block_fwd", L.F32, g, x.data_ptr(), m.data_ptr(), m.data_ptr(), m.data_ptr(), m.data_ptr(),
               None, 2, y.data_ptr(), L.F32, torch.cuda.current_stream().cuda_stream)
