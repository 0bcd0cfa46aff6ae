"""Determinism probe of the attention forward: the same call three times
(plain and keep-bit entry points, p = 0.1 and 0) must give bit-identical o."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hvit_amd_loader  # noqa: E402

l = hvit_amd_loader.load()._lib
B, N, H = 32, 256, 8
hd, D = 64, H * 64
torch.manual_seed(0)
qkv = (torch.randn(B * N, 3 * D, device="cuda") * 0.7).to(torch.bfloat16)
kb = torch.zeros(l.lib().hvit_mhsa_keep_bits_elems(B, N, H), dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for p in (0.1, 0.0):
    dr = l.dropout(p, 99, 31)
    res = []
    for rep in range(4):
        o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B, H, N, device="cuda")
        l.call("hvit_mhsa_fwd_kb", l.BF16, qkv.data_ptr(), B, N, H, hd, hd ** -0.5, dr, o.data_ptr(), lse.data_ptr(),
               kb.data_ptr() if rep % 2 else None, st)
        res.append(o)
    torch.cuda.synchronize()
    print(os.environ.get("HVIT_LIB", "libhvit.so"), f"p={p}",
          [int((res[0] != r).sum()) for r in res[1:]], flush=True)

# backward: the same call repeated
go = torch.randn(B * N, D, device="cuda").to(torch.bfloat16)
dr = l.dropout(0.1, 99, 31)
o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B, H, N, device="cuda")
l.call("hvit_mhsa_fwd_kb", l.BF16, qkv.data_ptr(), B, N, H, hd, hd ** -0.5, dr, o.data_ptr(), lse.data_ptr(),
       kb.data_ptr(), st)
res = []
for rep in range(4):
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, H, N, device="cuda")
    l.call("hvit_mhsa_bwd_kb", l.BF16, qkv.data_ptr(), o.data_ptr(), go.data_ptr(), lse.data_ptr(), B, N, H, hd,
           hd ** -0.5, dr, kb.data_ptr() if rep % 2 else None, dqkv.data_ptr(), delta.data_ptr(), st)
    res.append(dqkv)
torch.cuda.synchronize()
print("bwd", [int((res[0] != r).sum()) for r in res[1:]], flush=True)
