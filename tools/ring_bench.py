"""A/B of the bf16 ViT linear GEMMs across pipeline configurations
(hvit_gemm_tune: 0 = gemm.h two-stage kernels, 1-4 = gemm_ring.h LDS-ring
configurations), B=32 x 256 tokens, with the model's fused epilogues.  Every
configuration's output is checked against configuration 0's (same bf16
operands; differences are accumulation order only).  HIP-event timing,
configurations interleaved round by round in one process.

    python tools/ring_bench.py [cfgs=0,1,2,3,4] [rounds=3]
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
M, D, HID = 8192, 512, 2048


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


KEEP = []  # every tensor a launch reads through a raw pointer stays alive


def r(*shape):
    t = (torch.randn(*shape, device=DEV) * 0.5).to(BF)
    KEEP.append(t)
    return t


def cases():
    g = torch.Generator(device="cpu").manual_seed(0)
    out = []
    # forward kinds (hybrid_vit: qkv STORE+bias, proj RESID, fc1 GELU_DUAL, fc2 RESID)
    x, wq, bq = r(M, D), r(3 * D, D), torch.randn(3 * D, device=DEV)
    yq = torch.empty(M, 3 * D, device=DEV, dtype=BF)
    out.append(("fwd qkv", 2 * M * 3 * D * D, lambda: L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), wq.data_ptr(),
                                                               bq.data_ptr(), M, 3 * D, D, yq.data_ptr(), L.BF16, None,
                                                               s()), [yq]))
    o, wp, bp = r(M, D), r(D, D), torch.randn(D, device=DEV)
    res = torch.randn(M, D, device=DEV)
    rs = torch.rand(32, device=DEV) + 0.5
    KEEP.extend([res, rs, bq])
    x1 = torch.empty(M, D, device=DEV)
    ep_p = HF.epilogue(drop=L.dropout(0.1, 77, 301), resid=res, rowscale=rs, rps=256)
    out.append(("fwd proj+resid", 2 * M * D * D, lambda: L.call("hvit_linear_fwd", L.BF16, o.data_ptr(), wp.data_ptr(),
                                                                 bp.data_ptr(), M, D, D, x1.data_ptr(), L.F32, ep_p,
                                                                 s()), [x1]))
    w1, b1 = r(HID, D), torch.randn(HID, device=DEV)
    h = torch.empty(M, HID, device=DEV, dtype=BF)
    a = torch.empty(M, HID, device=DEV, dtype=BF)
    ep_1 = HF.epilogue(act=L.ACT_GELU_DUAL, out2=a, drop=L.dropout(0.1, 78, 302))
    out.append(("fwd fc1+gelu", 2 * M * HID * D, lambda: L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w1.data_ptr(),
                                                                 b1.data_ptr(), M, HID, D, h.data_ptr(), L.BF16, ep_1,
                                                                 s()), [h, a]))
    aa, w2, b2 = r(M, HID), r(D, HID), torch.randn(D, device=DEV)
    x2 = torch.empty(M, D, device=DEV)
    ep_2 = HF.epilogue(drop=L.dropout(0.1, 79, 303), resid=res, rowscale=rs, rps=256)
    out.append(("fwd fc2+resid", 2 * M * D * HID, lambda: L.call("hvit_linear_fwd", L.BF16, aa.data_ptr(),
                                                                  w2.data_ptr(), b2.data_ptr(), M, D, HID,
                                                                  x2.data_ptr(), L.F32, ep_2, s()), [x2]))
    # probes: plain bf16 GEMMs big enough to fill every configuration's grid
    for KK in (512, 2048, 4096):
        xp, wpp = r(M, KK), r(HID, KK)
        yp = torch.empty(M, HID, device=DEV, dtype=BF)
        KEEP.extend([xp, wpp, yp])
        out.append((f"probe 8192x2048x{KK}", 2 * M * HID * KK,
                    lambda xp=xp, wpp=wpp, yp=yp, KK=KK: L.call("hvit_linear_fwd", L.BF16, xp.data_ptr(),
                                                                wpp.data_ptr(), None, M, HID, KK, yp.data_ptr(),
                                                                L.BF16, None, s()), [yp]))
    # data gradients (fc2: GELU backward + bias-grad column sums; others plain)
    g2 = r(M, D)
    dh = torch.empty(M, HID, device=DEV, dtype=BF)
    cs = torch.zeros((M // 64, HID), device=DEV)  # colsum partial rows (one per 64-row block)
    KEEP.extend([cs, h, a, b1, b2, bp])
    ep_g = HF.epilogue(act=L.ACT_GELU_BWD, aux=h, drop=L.dropout(0.1, 78, 302), colsum=cs)

    def fc2d():
        L.call("hvit_linear_dgrad", L.BF16, g2.data_ptr(), w2.data_ptr(), M, D, HID, dh.data_ptr(), L.BF16, ep_g, s())
    out.append(("dgrad fc2+geluB", 2 * M * D * HID, fc2d, [dh, cs]))
    dxn2 = torch.empty(M, D, device=DEV)
    out.append(("dgrad fc1", 2 * M * D * HID, lambda: L.call("hvit_linear_dgrad", L.BF16, dh.data_ptr(), w1.data_ptr(),
                                                              M, HID, D, dxn2.data_ptr(), L.F32, None, s()), [dxn2]))
    do = torch.empty(M, D, device=DEV, dtype=BF)
    out.append(("dgrad proj", 2 * M * D * D, lambda: L.call("hvit_linear_dgrad", L.BF16, g2.data_ptr(), wp.data_ptr(),
                                                             M, D, D, do.data_ptr(), L.BF16, None, s()), [do]))
    dq = r(M, 3 * D)
    dxn1 = torch.empty(M, D, device=DEV)
    out.append(("dgrad qkv", 2 * M * 3 * D * D, lambda: L.call("hvit_linear_dgrad", L.BF16, dq.data_ptr(),
                                                                wq.data_ptr(), M, 3 * D, D, dxn1.data_ptr(), L.F32, None,
                                                                s()), [dxn1]))
    # weight gradients (dw = dy^T x, f32)
    for name, dy, xx, N, K in (("wgrad fc2", g2, aa, D, HID), ("wgrad fc1", dh, x, HID, D), ("wgrad proj", g2, o, D, D),
                               ("wgrad qkv", dq, x, 3 * D, D)):
        holder = {}

        def wg(dy=dy, xx=xx, N=N, K=K, holder=holder):
            holder["dw"] = HF.linear_wgrad(L.BF16, dy, xx, M, N, K)
        wg()
        out.append((name, 2 * M * N * K, wg, holder))
        tk = torch.zeros(HF.wgrad_tickets(M, N, K), device=DEV)
        KEEP.append(tk)
        holder2 = {}

        def wgt(dy=dy, xx=xx, N=N, K=K, holder=holder2, tk=tk):
            holder["dw"] = HF.linear_wgrad(L.BF16, dy, xx, M, N, K, tickets=tk)
        wgt()
        out.append((name + " tk", 2 * M * N * K, wgt, holder2))
    return out


def outputs(o):
    return [t.clone() for t in (o if isinstance(o, list) else [o["dw"]])]


def main():
    args = dict(a.split("=") for a in sys.argv[1:])
    cfgs = [int(c) for c in args.get("cfgs", "0,1,2,3,4").split(",")]
    rounds = int(args.get("rounds", "3"))
    cs = cases()
    if "only" in args:
        cs = [c for c in cs if args["only"] in c[0]]
    check = args.get("check", "1") == "1"
    ref = {}
    times = {(n, c): [] for n, *_ in cs for c in cfgs}
    for rd in range(rounds):
        for c in cfgs:
            L.lib().hvit_gemm_tune(0, c)
            for name, fl, fn, outs in cs:
                if not check:
                    times[(name, c)].append(timeit(fn))
                    continue
                fn()
                torch.cuda.synchronize()
                got = outputs(outs)
                if name not in ref:
                    L.lib().hvit_gemm_tune(0, 0)
                    fn()
                    torch.cuda.synchronize()
                    ref[name] = outputs(outs)
                    L.lib().hvit_gemm_tune(0, c)
                    fn()
                    torch.cuda.synchronize()
                    got = outputs(outs)
                if rd == 0:
                    errs = []
                    for a_, b_ in zip(got, ref[name]):
                        d = (a_.float() - b_.float()).abs().max().item()
                        sc = b_.float().abs().max().item() + 1e-12
                        errs.append(d / sc)
                    print(f"check cfg {c} {name:18s} max|d|/max|ref| = {max(errs):.2e}", flush=True)
                times[(name, c)].append(timeit(fn))
    print()
    hdr = "".join(f"   cfg{c:d} us   TF/s" for c in cfgs)
    print(f"{'gemm':18s}{hdr}")
    for name, fl, *_ in cs:
        row = ""
        for c in cfgs:
            t = sorted(times[(name, c)])[len(times[(name, c)]) // 2]
            row += f"  {t:8.1f} {fl / t / 1e6:6.0f}"
        print(f"{name:18s}{row}", flush=True)
    L.lib().hvit_gemm_tune(0, 1)


if __name__ == "__main__":
    main()
