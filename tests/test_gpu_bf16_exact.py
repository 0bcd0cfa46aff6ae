"""GPU: the bf16 throughput path pinned as tightly as its arithmetic allows.

Every kernel below is fed operands that are already bf16, and its reference is
torch fp32 arithmetic on exactly those rounded operands (bf16 x bf16 products
are exact in f32), so the only legitimate difference is f32 accumulation
order.  The checks are ELEMENT-WISE:

* f32 outputs:  |out - ref| <= ACC * max|ref|               (ACC = 2e-5)
* bf16 outputs: |out - ref| <= 2^-8 |ref| + ACC * max|ref|  (half a bf16 ulp:
  the kernel rounds its f32 value once, to nearest even)

so one wrong element (a swizzle or stage-ordering slip in an LDS-DMA image, a
mis-placed epilogue row) fails the test, unlike a max-relative bar at 2e-2.
The linear shapes are the B=32 ViT ones (M = 8192 tokens), and each is run on
every GEMM pipeline the library can pick (hvit_gemm_tune: automatic, gemm.h's
kernels, the LDS-ring 128x128 / 256x256 / 128x64 configurations), with each
fused epilogue the model uses (bias, GELU_DUAL + dropout, residual + DropPath
scale + dropout, GELU backward + bias-grad column sums, split-K slabs reduced
in a second launch or in-kernel).  Convolutions run the production shape
classes of the encoder / decoder (LDS-DMA implicit im2col) with the gradient
rounded to bf16 before the reference sees it."""

import pytest
import torch
import torch.nn.functional as F

from conftest import keep_mask

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16
ACC = 2e-5
CFGS = [-1, 0, 2, 4, 5]  # automatic, gemm.h only, ring 128x128 / 256x256 / 128x64


@pytest.fixture(scope="module")
def env(hv):
    import sys

    torch.backends.cuda.matmul.allow_tf32 = False
    HF = sys.modules["hvit_amd.functional"]
    yield hv._lib, HF
    hv._lib.lib().hvit_gemm_tune(0, -1)


def s():
    return torch.cuda.current_stream().cuda_stream


def check_f32(out, ref, acc=ACC, what=""):
    out, ref = out.double(), ref.double()
    bound = acc * ref.abs().max().item() + 1e-30
    bad = ((out - ref).abs() > bound)
    n = int(bad.sum())
    assert n == 0, f"{what}: {n} of {ref.numel()} elements off (max |d| {(out - ref).abs().max().item():.3e}, " \
                   f"bound {bound:.3e})"


def check_bf16(out, ref, acc=ACC, what=""):
    out, ref = out.double(), ref.double()
    bound = ref.abs() * 2.0 ** -8 + acc * ref.abs().max().item() + 1e-30
    bad = (out - ref).abs() > bound
    n = int(bad.sum())
    assert n == 0, f"{what}: {n} of {ref.numel()} elements beyond half a bf16 ulp"


def rb(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(BF)


M, D, HID = 8192, 512, 2048


@pytest.mark.parametrize("cfg", CFGS)
def test_linear_fwd_kinds_exact(env, cfg):
    L, HF = env
    L.lib().hvit_gemm_tune(0, cfg)
    torch.manual_seed(1)
    x = rb(M, D)
    # qkv: bias, bf16 out
    w, b = rb(3 * D, D, scale=D ** -0.5), torch.randn(3 * D, device=DEV)
    y = torch.empty(M, 3 * D, device=DEV, dtype=BF)
    L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w.data_ptr(), b.data_ptr(), M, 3 * D, D, y.data_ptr(), L.BF16,
           None, s())
    ref = x.float() @ w.float().t() + b
    check_bf16(y, ref, what=f"qkv cfg {cfg}")
    # fc1: GELU_DUAL + dropout (h bf16, a = dropout(gelu(h)) bf16)
    w1, b1 = rb(HID, D, scale=D ** -0.5), torch.randn(HID, device=DEV)
    h = torch.empty(M, HID, device=DEV, dtype=BF)
    a = torch.empty(M, HID, device=DEV, dtype=BF)
    L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w1.data_ptr(), b1.data_ptr(), M, HID, D, h.data_ptr(), L.BF16,
           HF.epilogue(act=L.ACT_GELU_DUAL, out2=a, drop=L.dropout(0.1, 21, 302)), s())
    ref = x.float() @ w1.float().t() + b1
    check_bf16(h, ref, what=f"fc1 h cfg {cfg}")
    mask = torch.as_tensor(keep_mask(21, 302, M * HID, 0.1).reshape(M, HID), device=DEV)
    check_bf16(a, F.gelu(ref) * mask / 0.9, acc=1e-4, what=f"fc1 a cfg {cfg}")  # GELU approximation <= 1.5e-7
    # fc1 as the model runs it: GELU_DUAL_D keeps gelu'(h) for the backward
    L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w1.data_ptr(), b1.data_ptr(), M, HID, D, h.data_ptr(), L.BF16,
           HF.epilogue(act=L.ACT_GELU_DUAL_D, out2=a, drop=L.dropout(0.1, 21, 302)), s())
    hp = ref.clone().requires_grad_(True)
    F.gelu(hp).backward(torch.ones_like(hp))
    check_bf16(h, hp.grad, acc=1e-4, what=f"fc1 gelu'(h) cfg {cfg}")
    check_bf16(a, F.gelu(ref) * mask / 0.9, acc=1e-4, what=f"fc1 a (D) cfg {cfg}")
    # GELU_DUAL_DK (the model's default): the stored multiplier carries the dropout mask
    L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w1.data_ptr(), b1.data_ptr(), M, HID, D, h.data_ptr(), L.BF16,
           HF.epilogue(act=L.ACT_GELU_DUAL_DK, out2=a, drop=L.dropout(0.1, 21, 302)), s())
    check_bf16(h, hp.grad * mask / 0.9, acc=1e-4, what=f"fc1 keep * gelu'(h) cfg {cfg}")
    check_bf16(a, F.gelu(ref) * mask / 0.9, acc=1e-4, what=f"fc1 a (DK) cfg {cfg}")
    # proj and fc2: f32 residual + DropPath row scale * dropout(v + b)
    res = torch.randn(M, D, device=DEV)
    rs = torch.rand(32, device=DEV) + 0.5
    for name, K in (("proj", D), ("fc2", HID)):
        xa = rb(M, K)
        wk, bk = rb(D, K, scale=K ** -0.5), torch.randn(D, device=DEV)
        out = torch.empty(M, D, device=DEV)
        L.call("hvit_linear_fwd", L.BF16, xa.data_ptr(), wk.data_ptr(), bk.data_ptr(), M, D, K, out.data_ptr(), L.F32,
               HF.epilogue(drop=L.dropout(0.1, 22, 303), resid=res, rowscale=rs, rps=256), s())
        mk = torch.as_tensor(keep_mask(22, 303, M * D, 0.1).reshape(M, D), device=DEV)
        v = (xa.float() @ wk.float().t() + bk) * mk / 0.9
        check_f32(out, res + rs.repeat_interleave(256)[:, None] * v, what=f"{name} cfg {cfg}")


@pytest.mark.parametrize("cfg", CFGS)
def test_linear_dgrad_kinds_exact(env, cfg):
    L, HF = env
    L.lib().hvit_gemm_tune(0, cfg)
    torch.manual_seed(2)
    # fc2 dgrad: dh = dropout_mask * gelu'(h) * (g2 W2), bf16 out, + bias-grad column sums
    g2 = rb(M, D)
    w2 = rb(D, HID, scale=D ** -0.5)
    h = rb(M, HID)
    dh = torch.empty(M, HID, device=DEV, dtype=BF)
    # colsum: one partial row per 64-row block (deterministic, no atomics), NaN-poisoned
    # so a row the epilogue fails to write shows up
    csr = torch.full((M // 64, HID), float("nan"), device=DEV)
    L.call("hvit_linear_dgrad", L.BF16, g2.data_ptr(), w2.data_ptr(), M, D, HID, dh.data_ptr(), L.BF16,
           HF.epilogue(act=L.ACT_GELU_BWD, aux=h, drop=L.dropout(0.1, 23, 304), colsum=csr), s())
    cs = csr.sum(0)
    hp = h.float().requires_grad_(True)
    F.gelu(hp).backward(torch.ones_like(hp))
    mk = torch.as_tensor(keep_mask(23, 304, M * HID, 0.1).reshape(M, HID), device=DEV)
    ref = (g2.float() @ w2.float()) * mk / 0.9 * hp.grad
    check_bf16(dh, ref, acc=1e-4, what=f"fc2 dgrad cfg {cfg}")
    check_f32(cs, ref.sum(0), acc=1e-4, what=f"fc2 dgrad colsum cfg {cfg}")
    # the model's form: MUL_AUX with the stored gelu'(h) (bf16) as the multiplier
    gd = hp.grad.to(BF)
    csr.fill_(float("nan"))
    L.call("hvit_linear_dgrad", L.BF16, g2.data_ptr(), w2.data_ptr(), M, D, HID, dh.data_ptr(), L.BF16,
           HF.epilogue(act=L.ACT_MUL_AUX, aux=gd, drop=L.dropout(0.1, 23, 304), colsum=csr), s())
    cs = csr.sum(0)
    ref = (g2.float() @ w2.float()) * mk / 0.9 * gd.float()
    check_bf16(dh, ref, what=f"fc2 dgrad MUL_AUX cfg {cfg}")
    check_f32(cs, ref.sum(0), acc=1e-4, what=f"fc2 dgrad MUL_AUX colsum cfg {cfg}")
    # with GELU_DUAL_DK's multiplier (mask folded in): MUL_AUX without a dropout
    gk = (hp.grad * mk / 0.9).to(BF)
    csr.fill_(float("nan"))
    L.call("hvit_linear_dgrad", L.BF16, g2.data_ptr(), w2.data_ptr(), M, D, HID, dh.data_ptr(), L.BF16,
           HF.epilogue(act=L.ACT_MUL_AUX, aux=gk, colsum=csr), s())
    cs = csr.sum(0)
    ref = (g2.float() @ w2.float()) * gk.float()
    check_bf16(dh, ref, what=f"fc2 dgrad MUL_AUX (DK) cfg {cfg}")
    check_f32(cs, ref.sum(0), acc=1e-4, what=f"fc2 dgrad MUL_AUX (DK) colsum cfg {cfg}")
    # fc1 / qkv dgrad (f32 out), proj dgrad (bf16 out)
    for name, N, K, odt in (("fc1", HID, D, L.F32), ("qkv", 3 * D, D, L.F32), ("proj", D, D, L.BF16)):
        dy = rb(M, N)
        w = rb(N, K, scale=N ** -0.5)
        dx = torch.empty(M, K, device=DEV, dtype=torch.float32 if odt == L.F32 else BF)
        L.call("hvit_linear_dgrad", L.BF16, dy.data_ptr(), w.data_ptr(), M, N, K, dx.data_ptr(), odt, None, s())
        ref = dy.float() @ w.float()
        (check_f32 if odt == L.F32 else check_bf16)(dx, ref, what=f"{name} dgrad cfg {cfg}")


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("N,K", [(D, HID), (HID, D), (D, D), (3 * D, D)])
def test_linear_wgrad_exact(env, cfg, N, K):
    L, HF = env
    L.lib().hvit_gemm_tune(0, cfg)
    torch.manual_seed(3)
    dy, x = rb(M, N), rb(M, K)
    ref = dy.float().t() @ x.float()
    dw = HF.linear_wgrad(L.BF16, dy, x, M, N, K)
    check_f32(dw, ref, what=f"wgrad {N}x{K} cfg {cfg}")
    tk = torch.zeros(HF.wgrad_tickets(M, N, K), device=DEV)
    for rep in range(2):  # the tickets are left zeroed for the next call
        dw = HF.linear_wgrad(L.BF16, dy, x, M, N, K, tickets=tk)
        check_f32(dw, ref, what=f"wgrad {N}x{K} cfg {cfg} in-kernel reduction (call {rep})")
    torch.cuda.synchronize()
    assert int(tk.count_nonzero()) == 0


@pytest.mark.parametrize("cfg", [-1, 0])
@pytest.mark.parametrize("N,K", [(D, HID), (HID, D), (D, D), (3 * D, D)])
def test_linear_wgrad_deferred_side_job(env, cfg, N, K):
    """hvit_linear_wgrad_defer leaves the split-K slabs; the next linear
    launch's epilogue side job sums them: dw bit-identical to the two-launch
    hvit_linear_wgrad, and the carrying dgrad's own output unchanged (fwd and
    dgrad carriers; also the M = 0 carrier, which runs the sum as its own
    launch)."""
    L, HF = env
    L.lib().hvit_gemm_tune(0, cfg)
    torch.manual_seed(4)
    dy, x = rb(M, N), rb(M, K)
    want = HF.linear_wgrad(L.BF16, dy, x, M, N, K)
    g, w = rb(M, D), rb(D, D, scale=D ** -0.5)
    out_ref = torch.empty(M, D, device=DEV, dtype=torch.float32)
    L.call("hvit_linear_dgrad", L.BF16, g.data_ptr(), w.data_ptr(), M, D, D, out_ref.data_ptr(), L.F32, None, s())
    for carrier in ("dgrad", "fwd", "empty"):
        dw, job = HF.linear_wgrad_deferred(L.BF16, dy, x, M, N, K)
        out = torch.empty_like(out_ref)
        if carrier == "dgrad":
            L.call("hvit_linear_dgrad", L.BF16, g.data_ptr(), w.data_ptr(), M, D, D, out.data_ptr(), L.F32,
                   HF.epilogue(side=job), s())
            assert torch.equal(out, out_ref)
        elif carrier == "fwd":
            L.call("hvit_linear_fwd", L.BF16, g.data_ptr(), w.data_ptr(), None, M, D, D, out.data_ptr(), L.F32,
                   HF.epilogue(side=job), s())
        else:
            L.call("hvit_linear_fwd", L.BF16, g.data_ptr(), w.data_ptr(), None, 0, D, D, out.data_ptr(), L.F32,
                   HF.epilogue(side=job), s())
        torch.cuda.synchronize()
        assert job.job.n in (0, N * K)
        assert torch.equal(dw, want), f"{carrier}: {(dw - want).abs().max().item()}"
    # a deferred weight gradient carrying another one's slabs (the model's
    # attention bias partials ride on the qkv weight gradient this way)
    dw1, j1 = HF.linear_wgrad_deferred(L.BF16, dy, x, M, N, K)
    dw2, j2 = HF.linear_wgrad_deferred(L.BF16, dy, x, M, N, K, side=j1)
    L.call("hvit_linear_dgrad", L.BF16, g.data_ptr(), w.data_ptr(), M, D, D, out.data_ptr(), L.F32,
           HF.epilogue(side=j2), s())
    torch.cuda.synchronize()
    assert torch.equal(dw1, want) and torch.equal(dw2, want)


@pytest.mark.parametrize("M,N,K", [(8192, 256, 512), (32768, 128, 128), (131072, 64, 64), (1000, 64, 128)])
def test_linear_wgrad_bias_deferred_side_job(env, M, N, K):
    """hvit_linear_wgrad_bias_defer (the head and skip projections' weight and
    bias gradients): the tall-skinny kernel's [dw | db] slabs summed by the next
    data-gradient launch's epilogue side job (HeadFn / SkipFn backward), and
    that launch's own output unchanged; dw and db element-wise at the
    accumulation-order bar (the slab sum's order differs from the two-launch
    hvit_linear_wgrad's), and bit-identical to the same job run by
    hvit_sum_slabs_strided (splits 4 / 32 / 128 / 512: both epi_side forms)."""
    L, HF = env
    torch.manual_seed(6)
    dy, x = rb(M, N), rb(M, K)
    g, w = rb(M, N), rb(N, K, scale=N ** -0.5)
    out_ref = torch.empty(M, K, device=DEV, dtype=torch.float32)
    L.call("hvit_linear_dgrad", L.BF16, g.data_ptr(), w.data_ptr(), M, N, K, out_ref.data_ptr(), L.F32, None, s())
    dw, db, job = HF.linear_wgrad_bias_deferred(L.BF16, dy, x, M, N, K)
    assert job is not None and job.job.n == N * K + N
    out = torch.empty_like(out_ref)
    L.call("hvit_linear_dgrad", L.BF16, g.data_ptr(), w.data_ptr(), M, N, K, out.data_ptr(), L.F32,
           HF.epilogue(side=job), s())
    # the job run as a launch of its own (side-stream form): the carried order, bit for bit
    dw2, db2, job2 = HF.linear_wgrad_bias_deferred(L.BF16, dy, x, M, N, K)
    j = job2.job
    L.call("hvit_sum_slabs_strided", j.src, j.splits, j.stride, j.n, j.dst, s())
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref)
    check_f32(dw, dy.float().t() @ x.float(), what=f"deferred small wgrad {M}x{N}x{K}")
    check_f32(db, dy.float().sum(0), what=f"deferred small wgrad bias {M}x{N}x{K}")
    assert torch.equal(dw2, dw) and torch.equal(db2, db)


@pytest.mark.parametrize("M,N,K", [(2048, 256, 512), (8192, 256, 256), (32768, 128, 128), (131072, 64, 64),
                                   (1000, 64, 128)])
def test_linear_wgrad_small_with_bias_exact(env, M, N, K):
    """The tall-skinny weight gradients of the step (head, skip projections:
    csrc/wgrad_small.hip) with the bias gradient, element-wise."""
    L, HF = env
    torch.manual_seed(5)
    dy, x = rb(M, N), rb(M, K)
    dw, db = HF.linear_wgrad(L.BF16, dy, x, M, N, K, bias=True)
    check_f32(dw, dy.float().t() @ x.float(), what=f"small wgrad {M}x{N}x{K}")
    check_f32(db, dy.float().sum(0), what=f"small wgrad bias {M}x{N}x{K}")
    dw2 = HF.linear_wgrad(L.BF16, dy, x, M, N, K)
    check_f32(dw2, dy.float().t() @ x.float(), what=f"small wgrad (no bias) {M}x{N}x{K}")


CONV_PROD = [
    # N, Hs, Ws, C1, C2, U, Cout: the model's LDS-DMA implicit-im2col shape classes
    (4, 128, 128, 64, 0, 1, 128),   # enc1
    (4, 64, 64, 128, 0, 1, 256),    # enc2
    (8, 16, 16, 256, 256, 1, 256),  # dec0 (decoder concat)
    (8, 16, 16, 256, 128, 2, 128),  # dec1 (x2 upsample + concat)
    (8, 32, 32, 128, 64, 2, 64),    # dec2
]


@pytest.mark.parametrize("case", CONV_PROD)
def test_conv3x3_bf16_exact(env, case):
    L, HF = env
    torch.manual_seed(4)
    N, Hs, Ws, C1, C2, U, Cout = case
    x1 = rb(N, Hs, Ws, C1)
    x2 = rb(N, Hs, Ws, C2) if C2 else None
    w = torch.randn(Cout, C1 + C2, 3, 3, device=DEV) / ((C1 + C2) * 9) ** 0.5
    wq = w.to(BF).float()
    xr = torch.cat([x1, x2], 3) if C2 else x1
    xr = xr.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    xu = F.interpolate(xr, scale_factor=U, mode="nearest") if U > 1 else xr
    wr = wq.clone().requires_grad_(True)
    ref = F.conv2d(xu, wr, None, 1, 1)
    H, W = Hs * U, Ws * U
    g = HF.geom(x1, C1, x2, C2, N, Hs, Ws, U, 3, 1, 1, Cout)
    wp = HF.pack_conv(w, 0, L.BF16)
    z = torch.empty(N, H, W, Cout, device=DEV)
    L.call("hvit_conv_fwd", L.BF16, g, wp.data_ptr(), None, z.data_ptr(), L.F32, None, None, s())
    check_f32(z.permute(0, 3, 1, 2), ref, what="conv fwd")
    gz = torch.randn_like(ref).to(BF)  # the bf16 gradient both sides see
    ref.backward(gz.float())
    dz = gz.permute(0, 2, 3, 1).contiguous()
    dw = HF.conv_wgrad(L.BF16, g, dz, w.shape)
    # the torch-layout entry (fused slab sum + unpack) against the packed one
    # followed by hvit_conv_weight_unpack: bit-identical
    ws_n = L.lib().hvit_conv_wgrad_workspace(g)
    ws = torch.empty(max(ws_n, 1), device=DEV)
    dwp = torch.empty(w.numel(), device=DEV)
    L.call("hvit_conv_wgrad", L.BF16, g, dz.data_ptr(), dwp.data_ptr(), ws.data_ptr(), ws_n, s())
    assert torch.equal(dw, HF.unpack_conv(dwp, w.shape))
    check_f32(dw, wr.grad, what="conv wgrad")
    wd = HF.pack_conv(w, 1, L.BF16)
    du = torch.empty(N, H, W, C1 + C2, device=DEV)
    L.call("hvit_conv_dgrad", L.BF16, g, dz.data_ptr(), wd.data_ptr(), du.data_ptr(), L.F32, s())
    # gradient w.r.t. the (upsampled, concatenated) conv input
    xu2 = xu.detach().requires_grad_(True)
    F.conv2d(xu2, wq, None, 1, 1).backward(gz.float())
    check_f32(du.permute(0, 3, 1, 2), xu2.grad, what="conv dgrad")
