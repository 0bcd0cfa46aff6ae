"""Time the grouped weight-gradient launch (hvit_linear_wgrad_group) on the
B=32 ViT shapes: `layers` blocks' qkv / proj / fc1 / fc2 dW over M tokens in
one launch, graph-replayed; prints us per launch, TFLOP/s and the MFMA-peak
fraction.  Under rocprofv3 (kernel trace / PMC passes) it is the kernel's
isolated loop.

    python tools/wgrad_group_probe.py [layers=6] [M=8192] [D=512] [reps=20] [cfg=0]
"""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
L = hv._lib
DEV = "cuda"
BF = torch.bfloat16


def main():
    args = dict(a.split("=") for a in sys.argv[1:])
    layers = int(args.get("layers", "6"))
    M = int(args.get("M", "8192"))
    D = int(args.get("D", "512"))
    reps = int(args.get("reps", "20"))
    cfg = int(args.get("cfg", "0"))  # hvit_gemm_tune(7, cfg): tile configuration
    same = int(args.get("same", "0"))  # 1: every block's problems read the same operands (L2-resident ceiling)
    L.lib().hvit_gemm_tune(7, cfg)
    hid = 4 * D
    g = torch.Generator(device=DEV).manual_seed(0)
    keep, probs, flops = [], [], 0.0
    first = {}
    for _ in range(layers):
        for n, k in ((D, hid), (hid, D), (D, D), (3 * D, D)):
            if same and (n, k) in first:
                dy, x = first[(n, k)]
            else:
                dy = (torch.randn(M, n, device=DEV, generator=g) * 0.5).to(BF)
                x = (torch.randn(M, k, device=DEV, generator=g) * 0.5).to(BF)
                first[(n, k)] = (dy, x)
            dw = torch.empty(n, k, device=DEV)
            keep += [dy, x, dw]
            probs.append(L.WgradProb(dy.data_ptr(), n, x.data_ptr(), k, dw.data_ptr(), n, k))
            flops += 2.0 * M * n * k
    arr = (L.WgradProb * len(probs))(*probs)
    ws = torch.empty(int(L.lib().hvit_linear_wgrad_group_ws()), device=DEV)
    tk = torch.zeros(int(L.lib().hvit_linear_wgrad_group_tickets()), dtype=torch.int32, device=DEV)

    def launch():
        L.call("hvit_linear_wgrad_group", L.BF16, M, arr, len(probs), ws.data_ptr(), ws.numel(), tk.data_ptr(),
               tk.numel(), torch.cuda.current_stream().cuda_stream)

    launch()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            launch()
    gr.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    ts.sort()
    us = ts[2]
    tf = flops / us / 1e6
    print(f"cfg={cfg} same={same} layers={layers} M={M} D={D} problems={len(probs)}: {us:.1f} us per launch, {flops / 1e9:.1f} GFLOP, "
          f"{tf:.0f} TFLOP/s, frac {tf / 2500:.3f}", flush=True)


if __name__ == "__main__":
    main()
