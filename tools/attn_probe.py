"""Attention v2 forward / backward probe: per-shape error against an fp32
torch reference (by query block and d-block), repeat-call equality, and the
keep-bit vs re-hash equality of o, lse and dqkv."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
l = hv._lib
DEV = "cuda"
S = lambda: torch.cuda.current_stream().cuda_stream


def ref(qkv, B, N, H, hd):
    q, k, v = qkv.float().view(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    a = ((q @ k.transpose(-2, -1)) * hd ** -0.5).softmax(-1)
    return (a @ v).transpose(1, 2).reshape(B * N, H * hd)


def fwd(qkv, B, N, H, dr, kb=None):
    D = H * 64
    o = torch.full((B * N, D), float("nan"), device=DEV, dtype=torch.bfloat16)
    lse = torch.full((B, H, N), float("nan"), device=DEV)
    if kb is None:
        l.call("hvit_mhsa_fwd", l.BF16, qkv.data_ptr(), B, N, H, 64, 0.125, dr, o.data_ptr(), lse.data_ptr(), None, S())
    else:
        l.call("hvit_mhsa_fwd_kb", l.BF16, qkv.data_ptr(), B, N, H, 64, 0.125, dr, o.data_ptr(), lse.data_ptr(),
               kb.data_ptr(), S())
    return o, lse


def bwd(qkv, o, go, lse, B, N, H, dr, kb=None):
    dqkv = torch.full_like(qkv, float("nan"))
    delta = torch.empty(B, H, N, device=DEV)
    if kb is None:
        l.call("hvit_mhsa_bwd", l.BF16, qkv.data_ptr(), o.data_ptr(), go.data_ptr(), lse.data_ptr(), B, N, H, 64,
               0.125, dr, dqkv.data_ptr(), delta.data_ptr(), S())
    else:
        l.call("hvit_mhsa_bwd_kb", l.BF16, qkv.data_ptr(), o.data_ptr(), go.data_ptr(), lse.data_ptr(), B, N, H, 64,
               0.125, dr, kb.data_ptr(), dqkv.data_ptr(), delta.data_ptr(), S())
    return dqkv


for B, N, H in [(2, 256, 8), (2, 240, 8), (2, 300, 2), (2, 496, 8), (1, 512, 4), (2, 272, 2)]:
    torch.manual_seed(N)
    D = H * 64
    qkv = (torch.randn(B * N, 3 * D, device=DEV) * 0.7).to(torch.bfloat16)
    o, lse = fwd(qkv, B, N, H, None)
    r = ref(qkv, B, N, H, 64)
    err = (o.float() - r).abs()
    print(f"B={B} N={N} H={H}: fwd max err {err.max().item():.4g} (ref max {r.abs().max().item():.3g}), nan {torch.isnan(o.float()).sum().item()}")
    e4 = err.view(B, N, H, 4, 16).amax(dim=(0, 2, 4))  # [N, 4 d-blocks]
    bad = (e4 > 0.02 * r.abs().max()).nonzero()
    if len(bad):
        qs = sorted(set(bad[:, 0].tolist()))
        print("   bad queries", len(qs), qs[:8], "...", qs[-8:], " d-blocks", sorted(set(bad[:, 1].tolist())))
        eb = torch.nn.functional.pad(e4.amax(1), (0, (-N) % 16))
        print("   per 16-query block max err", [round(x, 3) for x in eb.view(-1, 16).amax(1).tolist()])
    reps = [fwd(qkv, B, N, H, None) for _ in range(4)]
    print("   repeat-equal o", all(torch.equal(reps[0][0], x[0]) for x in reps[1:]),
          "lse", all(torch.equal(reps[0][1], x[1]) for x in reps[1:]))
    dr = l.dropout(0.1, 99, 31)
    kb = torch.zeros(l.lib().hvit_mhsa_keep_bits_elems(B, N, H), dtype=torch.int32, device=DEV)
    go = torch.randn(B * N, D, device=DEV).to(torch.bfloat16)
    oa, la = fwd(qkv, B, N, H, dr)
    ob, lb = fwd(qkv, B, N, H, dr, kb)
    da = bwd(qkv, oa, go, la, B, N, H, dr)
    db = bwd(qkv, ob, go, lb, B, N, H, dr, kb)
    da2 = bwd(qkv, oa, go, la, B, N, H, dr)
    db2 = bwd(qkv, ob, go, lb, B, N, H, dr, kb)
    torch.cuda.synchronize()
    dd = (da.float() - db.float()).abs().view(B * N, 3, D).amax(dim=(0, 2))
    print("   kb vs rehash: o", torch.equal(oa, ob), "lse", torch.equal(la, lb), "dqkv", torch.equal(da, db),
          "dq/dk/dv maxdiff", [round(x, 5) for x in dd.tolist()],
          "repeat rehash", torch.equal(da, da2), "repeat kb", torch.equal(db, db2))
