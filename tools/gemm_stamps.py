"""Where a GEMM workgroup spends its time (diagnostic build libhvit_stamps.so,
-DHVIT_GEMM_STAMPS): per-workgroup wall-clock stamps at start, after the K
loop and at exit.  Run with HVIT_LIB=libhvit_stamps.so."""

import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib
BF = torch.bfloat16
TICK_US = 0.01  # s_memrealtime: 100 MHz


def stamps(nblk):
    buf = (C.c_ulonglong * (nblk * 4))()
    assert L.lib().hvit_debug_gemm_stamps(buf, nblk * 4) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(nblk, 4).astype(np.float64)


def probe(M, N, K, tag, epi=None):
    x = torch.randn(M, K, device="cuda").to(BF)
    w = torch.randn(N, K, device="cuda").to(BF)
    b = torch.zeros(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=BF)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        L.call("hvit_linear_fwd", L.BF16, x.data_ptr(), w.data_ptr(), b.data_ptr(), M, N, K, y.data_ptr(), L.BF16,
               epi, st)
    torch.cuda.synchronize()
    nblk = (M // 128) * (N // 128)
    s = stamps(nblk)
    t0 = s[:, 0].min()
    start = (s[:, 0] - t0) * TICK_US
    loop = (s[:, 1] - s[:, 0]) * TICK_US
    epil = (s[:, 2] - s[:, 1]) * TICK_US
    end = (s[:, 2] - t0) * TICK_US
    print(f"{tag}: M={M} N={N} K={K} blocks={nblk}  span {end.max():.1f} us")
    print(f"   start  min/med/max {start.min():6.1f} {np.median(start):6.1f} {start.max():6.1f} us")
    print(f"   loop   min/med/max {loop.min():6.1f} {np.median(loop):6.1f} {loop.max():6.1f} us")
    print(f"   epilog min/med/max {epil.min():6.1f} {np.median(epil):6.1f} {epil.max():6.1f} us", flush=True)
    hist = np.histogram(start, bins=8)
    print("   start histogram:", list(hist[0]), [round(v, 1) for v in hist[1]])


def probe_wgrad(M, N, K, tag):
    """dw[N, K] = dy[M, N]^T x[M, K] (split-K slabs), stamps of the GEMM launch"""
    dy = torch.randn(M, N, device="cuda").to(BF)
    x = torch.randn(M, K, device="cuda").to(BF)
    dw = torch.empty(N, K, device="cuda")
    ws_n = L.lib().hvit_wgrad_workspace(M, N, K)
    ws = torch.empty(max(ws_n, 1), device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        L.call("hvit_linear_wgrad", L.BF16, dy.data_ptr(), x.data_ptr(), M, N, K, dw.data_ptr(), None,
               ws.data_ptr(), ws_n, st)
    torch.cuda.synchronize()
    splits = ws_n // (N * K + N) if ws_n else 1
    nblk = (N // 128) * (K // 128) * max(splits, 1)
    s = stamps(nblk)
    t0 = s[:, 0].min()
    loop = (s[:, 1] - s[:, 0]) * TICK_US
    epil = (s[:, 2] - s[:, 1]) * TICK_US
    end = (s[:, 2] - t0) * TICK_US
    print(f"{tag}: M={M} N={N} K={K} splits~{splits} blocks={nblk} span {end.max():.1f} us  "
          f"loop med {np.median(loop):.1f}  epilog med {np.median(epil):.1f} us", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "wgrad":
        for N_, K_ in [(512, 2048), (2048, 512), (512, 512), (1536, 512)]:
            probe_wgrad(8192, N_, K_, f"wgrad {N_}x{K_}")
        sys.exit(0)
    probe(8192, 2048, 512, "fc1 plain")
    probe(8192, 2048, 2048, "fc1 K=2048")
    probe(8192, 512, 512, "proj plain")
    a = torch.empty(8192, 2048, device="cuda", dtype=BF)
    probe(8192, 2048, 512, "fc1 gelu+drop", HF_epi := sys.modules["hvit_amd.functional"].epilogue(
        act=L.ACT_GELU_DUAL, out2=a, drop=L.dropout(0.1, 1, 1)))
