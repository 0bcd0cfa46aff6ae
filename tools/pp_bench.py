"""A/B of the persistent epilogue-overlapped GEMM (csrc/gemm_pp.hip) against the
ring / gemm.h kernels on the B=32 ViT shapes it serves: qkv forward (+bias),
fc1 forward (+bias, GELU, dropout: stores gelu'(h) and a), fc2 data gradient
(dropout x gelu'(h) backward, fc1 bias-grad column sums, a carried split-K
slab-sum side job).  hvit_gemm_tune(3, mode): 0 = the previous kernels, 1 =
256x128 tiles (8 waves), 2 = 128x128 (4 waves, two workgroups per CU).

Every mode's outputs are compared with mode 0's (same bf16 operands: the
accumulation order is the same k order, so they should agree bit for bit) and
with a torch fp32 reference of the same op; HIP-event timing with the modes
interleaved round by round in one process.

    python tools/pp_bench.py [modes=0,1,2] [rounds=5] [M=8192] [what=3]

what=W A/Bs the values `modes` of another hvit_gemm_tune knob W instead (the
persistent kernels off); the weight-gradient rows time the ring / gemm.h
weight-gradient kernels with their slab sums.
"""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib
HF = sys.modules["hvit_amd.functional"]
DEV = "cuda"
BF = torch.bfloat16
KEEP = []


def s():
    return L.stream_ptr()


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def r(*shape, scale=0.5):
    t = (torch.randn(*shape, device=DEV) * scale).to(BF)
    KEEP.append(t)
    return t


def gelu_ref(h):
    return 0.5 * h * (1.0 + torch.erf(h * 0.7071067811865476))


def gelu_grad_ref(h):
    cdf = 0.5 * (1.0 + torch.erf(h * 0.7071067811865476))
    return cdf + h * 0.3989422804014327 * torch.exp(-0.5 * h * h)


def cases(M, D=512, HID=2048):
    out = []
    # qkv forward: y = x W^T + b (bf16)
    x, wq, bq = r(M, D), r(3 * D, D, scale=0.05), torch.randn(3 * D, device=DEV)
    KEEP.append(bq)
    yq = torch.empty(M, 3 * D, device=DEV, dtype=BF)

    def ref_q():
        return [(x.float() @ wq.float().t() + bq)]
    out.append(("fwd qkv", 2 * M * 3 * D * D,
                lambda: L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), wq.data_ptr(), bq.data_ptr(), M, 3 * D, D,
                               yq.data_ptr(), L.BF16, None, s()), [yq], ref_q))
    # fc1 forward: gelu'(h) and a = dropout(gelu(h)) (no dropout in the torch check: p = 0 variant below)
    w1, b1 = r(HID, D, scale=0.05), torch.randn(HID, device=DEV) * 0.5
    KEEP.append(b1)
    gh = torch.empty(M, HID, device=DEV, dtype=BF)
    a = torch.empty(M, HID, device=DEV, dtype=BF)
    ep_1 = HF.epilogue(act=L.ACT_GELU_DUAL_D, out2=a, drop=L.dropout(0.1, 78, 302))
    out.append(("fwd fc1+gelu p.1", 2 * M * HID * D,
                lambda: L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w1.data_ptr(), b1.data_ptr(), M, HID, D,
                               gh.data_ptr(), L.BF16, ep_1, s()), [gh, a], None))
    gh0 = torch.empty(M, HID, device=DEV, dtype=BF)
    a0 = torch.empty(M, HID, device=DEV, dtype=BF)
    ep_10 = HF.epilogue(act=L.ACT_GELU_DUAL_D, out2=a0)

    def ref_1():
        h = x.float() @ w1.float().t() + b1
        return [gelu_grad_ref(h), gelu_ref(h)]
    out.append(("fwd fc1+gelu p0", 2 * M * HID * D,
                lambda: L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w1.data_ptr(), b1.data_ptr(), M, HID, D,
                               gh0.data_ptr(), L.BF16, ep_10, s()), [gh0, a0], ref_1))
    # fc2 data gradient: dh = (g2 W2) * keep * gelu'(h), colsum partial rows
    g2, w2 = r(M, D), r(D, HID, scale=0.05)
    dh = torch.empty(M, HID, device=DEV, dtype=BF)
    cs = torch.zeros((M // 64, HID), device=DEV)
    KEEP.extend([cs, gh, a, gh0])
    ep_g = HF.epilogue(act=L.ACT_MUL_AUX, aux=gh, drop=L.dropout(0.1, 78, 302), colsum=cs)
    out.append(("dgrad fc2+geluB p.1", 2 * M * D * HID,
                lambda: L.call("hvit_linear_dgrad", L.BF16, g2.data_ptr(), w2.data_ptr(), M, D, HID, dh.data_ptr(),
                               L.BF16, ep_g, s()), [dh, cs], None))
    dh0 = torch.empty(M, HID, device=DEV, dtype=BF)
    cs0 = torch.zeros((M // 64, HID), device=DEV)
    KEEP.extend([dh0, cs0])
    ep_g0 = HF.epilogue(act=L.ACT_MUL_AUX, aux=gh0, colsum=cs0)

    def ref_2():
        d = (g2.float() @ w2.float()) * gh0.float()
        return [d, d.sum(0)]
    out.append(("dgrad fc2+geluB p0", 2 * M * D * HID,
                lambda: L.call("hvit_linear_dgrad", L.BF16, g2.data_ptr(), w2.data_ptr(), M, D, HID, dh0.data_ptr(),
                               L.BF16, ep_g0, s()), [dh0, cs0], ref_2))
    # a conv-shaped dense GEMM (enc1 forward as a plain GEMM: M = 32 x 128 x 128 pixels, N = 128
    # channels, K = 64 x 9 taps; the real conv gathers A by implicit im2col)
    if os.environ.get("PP_CONVLIKE"):
        Mc = 32 * 128 * 128
        xc, wc = r(Mc, 576), r(128, 576, scale=0.05)
        yc = torch.empty(Mc, 128, device=DEV, dtype=BF)
        KEEP.append(yc)
        out.append(("convlike fwd", 2 * Mc * 128 * 576,
                    lambda: L.call("hvit_linear_fwd", L.BF16, xc.data_ptr(), wc.data_ptr(), None, Mc, 128, 576,
                                   yc.data_ptr(), L.BF16, None, s()), [yc], None))
    # N = 512 data gradients (dy [M, K] x W [K, 512]: qkv / proj in bf16, fc1 in f32 for the LN backward)
    for nm, k_, odt in (("dgrad qkv->512", 3 * D, L.BF16), ("dgrad proj->512", D, L.BF16), ("dgrad fc1->512", HID, L.F32)):
        dy_, w_ = r(M, k_), r(k_, D, scale=0.05)
        o_ = torch.empty(M, D, device=DEV, dtype=BF if odt == L.BF16 else torch.float32)
        KEEP.append(o_)

        def fd(dy_=dy_, w_=w_, k_=k_, o_=o_, odt=odt):
            L.call("hvit_linear_dgrad", L.BF16, dy_.data_ptr(), w_.data_ptr(), M, k_, D, o_.data_ptr(), odt, None, s())

        def rd(dy_=dy_, w_=w_):
            return [dy_.float() @ w_.float()]
        out.append((nm, 2 * M * k_ * D, fd, [o_], rd))
    # weight gradients (both operands k-major: the ring kernels' 128x128 / 128x64 forms + slab sums)
    for nm, n_, k_ in (("wgrad qkv", 3 * D, D), ("wgrad fc1", HID, D), ("wgrad fc2", D, HID), ("wgrad proj", D, D)):
        dy_, x_ = r(M, n_), r(M, k_)
        dw_ = torch.empty(n_, k_, device=DEV)
        KEEP.append(dw_)

        def fw(dy_=dy_, x_=x_, n_=n_, k_=k_, dw_=dw_):
            HF.linear_wgrad_now(L.BF16, dy_, x_, M, n_, k_, dest=dw_)

        def rw(dy_=dy_, x_=x_):
            return [dy_.float().t() @ x_.float()]
        out.append((nm, 2 * M * n_ * k_, fw, [dw_], rw))
    return out


def view(t):
    """The column-sum partial rows are compared through their column totals: how
    many rows a kernel fills with partials (and which it zeroes) is its own
    business, the slab sum that consumes them only needs the total."""
    return t.double().sum(0) if t.dtype == torch.float32 and t.dim() == 2 and t.shape[0] < 1024 else t


def rel(a_, b_):
    a_, b_ = view(a_), view(b_)
    d = (a_.double() - b_.double()).abs().max().item()
    return d / (b_.double().abs().max().item() + 1e-12)


def main():
    args = dict(a.split("=") for a in sys.argv[1:])
    modes = [int(c) for c in args.get("modes", "0,1,2").split(",")]
    rounds = int(args.get("rounds", "5"))
    M = int(args.get("M", "8192"))
    what = int(args.get("what", "3"))  # the hvit_gemm_tune knob the modes set
    if what != 3:
        L.lib().hvit_gemm_tune(3, 0)
    old = L.lib().hvit_gemm_tune(what, modes[0])
    cs = cases(M)
    ref = {}
    times = {(n, c): [] for n, *_ in cs for c in modes}
    bad = 0
    for rd in range(rounds):
        for c in modes:
            L.lib().hvit_gemm_tune(what, c)
            for name, fl, fn, outs, tref in cs:
                if rd == 0:
                    for t in outs:
                        t.fill_(float("nan")) if t.is_floating_point() else None
                    fn()
                    torch.cuda.synchronize()
                    got = [t.clone() for t in outs]
                    if c == modes[0]:
                        ref[name] = got
                    eq = [torch.equal(a_, b_) for a_, b_ in zip(got, ref[name])]
                    e_mode = max(rel(a_, b_) for a_, b_ in zip(got, ref[name]))
                    per = [f"{rel(a_, b_):.1e}" for a_, b_ in zip(got, ref[name])]
                    msg = f"check mode {c} {name:22s} vs mode {modes[0]}: bitwise {eq} max|d|/max = {e_mode:.2e} {per}"
                    if tref is not None:
                        rs = tref()
                        e_t = max(rel(a_, b_) for a_, b_ in zip(got, rs))
                        msg += f"   vs torch fp32: {e_t:.2e}"
                        if e_t > 2e-2:
                            bad += 1
                    finite = all(torch.isfinite(t).all().item() for t in got)
                    if not finite:
                        msg += "   NON-FINITE"
                        bad += 1
                    print(msg, flush=True)
                times[(name, c)].append(timeit(fn))
    print()
    hdr = "".join(f"   mode{c:d} us   TF/s" for c in modes)
    print(f"{'gemm':22s}{hdr}")
    for name, fl, *_ in cs:
        row = ""
        for c in modes:
            t = sorted(times[(name, c)])[len(times[(name, c)]) // 2]
            row += f"  {t:9.1f} {fl / t / 1e6:6.0f}"
        print(f"{name:22s}{row}", flush=True)
    L.lib().hvit_gemm_tune(what, old)
    if bad:
        print(f"FAILED checks: {bad}")
        sys.exit(1)


if __name__ == "__main__":
    main()
