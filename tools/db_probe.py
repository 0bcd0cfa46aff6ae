"""hvit_mhsa_bwd_db partial bias rows (non-v2 shapes, hd 16): eager vs the
same calls captured in a CUDA graph and replayed, against a column reduction."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hvit_amd_loader  # noqa: E402

l = hvit_amd_loader.load()._lib
for (B, N, H, hd) in ((2, 12, 4, 16), (2, 256, 8, 64), (2, 300, 2, 64)):
    D = H * hd
    torch.manual_seed(0)
    qkv = (torch.randn(B * N, 3 * D, device="cuda") * 0.7).to(torch.bfloat16)
    go = torch.randn(B * N, D, device="cuda").to(torch.bfloat16)
    o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device="cuda")
    dr = l.dropout(0.1, 5, 7)
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    l.call("hvit_mhsa_fwd", l.BF16, qkv.data_ptr(), B, N, H, hd, hd ** -0.5, dr, o.data_ptr(), lse.data_ptr(), None,
           st())
    rows = l.lib().hvit_mhsa_bias_rows(l.BF16, B, N, H, hd)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, H, N, device="cuda")
    parts = torch.empty(rows, 3 * D, device="cuda")
    db = torch.empty(3 * D, device="cuda")

    def run():
        l.call("hvit_mhsa_bwd_db", l.BF16, qkv.data_ptr(), o.data_ptr(), go.data_ptr(), lse.data_ptr(), B, N, H, hd,
               hd ** -0.5, dr, None, dqkv.data_ptr(), delta.data_ptr(), parts.data_ptr(), st())
        l.call("hvit_sum_slabs_strided", parts.data_ptr(), rows, 3 * D, 3 * D, db.data_ptr(), st())
    run()
    torch.cuda.synchronize()
    eager = db.clone()
    ref = dqkv.float().sum(0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    db.fill_(-1)
    with torch.cuda.graph(g):
        run()
    g.replay()
    torch.cuda.synchronize()
    print((B, N, H, hd), "rows", rows, "eager vs ref", (eager - ref).abs().max().item(), "graph vs ref",
          (db - ref).abs().max().item(), "ref max", ref.abs().max().item(), flush=True)
