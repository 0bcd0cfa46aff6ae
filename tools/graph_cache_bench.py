"""BASELINE config 3/4's train step on VoiceBank-shaped batches through the
per-shape graph cache (…_amd/train_step.py GraphedTrainStep; SURVEY §8(f)
rank 3): B = 32 spectrograms [32, 1, 257, T] whose T changes from batch to
batch, as collate_fn's right-padding produces (data/dataset.py:297-347).
Shapes T in {240, 251, 300} (2 s, 2 s, 2.4 s clips: N = 240 / 240 / 288
tokens) are visited in rotation; after each shape's warm-up every step is a
replay of that shape's captured step.  Reports per shape the replayed and the
eager ms/step and frames/s (frames = B x T), and the cache counters.

    python tools/graph_cache_bench.py [steps=12] [B=32]
"""

import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hvit_amd_loader  # noqa: E402

hv = hvit_amd_loader.load()
import importlib  # noqa: E402

ts = importlib.import_module("hvit_amd.train_step")


def main():
    args = dict(a.split("=") for a in sys.argv[1:])
    steps = int(args.get("steps", "12"))
    B = int(args.get("B", "32"))
    Ts = [240, 251, 300]
    torch.manual_seed(0)
    model = hv.HybridViT(precision="bf16").cuda().train()
    opt = hv.FusedAdamW(model.parameters(), lr=1e-4, weight_decay=0.01, max_grad_norm=1.0, capturable=True)
    crit = hv.CombinedLoss()
    step = ts.GraphedTrainStep(model, crit, opt, max_graphs=4, warmup=2)
    g = torch.Generator(device="cuda").manual_seed(1)
    data = {T: (torch.rand(B, 1, 257, T, device="cuda", generator=g), torch.rand(B, 1, 257, T, device="cuda", generator=g))
            for T in Ts}
    # warm-up + capture of every shape
    for _ in range(3):
        for T in Ts:
            step(*data[T])
    torch.cuda.synchronize()
    res = {}
    for T in Ts:
        x, t = data[T]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(steps):
            loss = step(x, t)
        ev[1].record()
        ev[1].synchronize()
        ms = ev[0].elapsed_time(ev[1]) / steps
        # the same steps eagerly (no graph), for reference
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            l2 = crit(model(x), t)
            l2.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
        e1.record()
        e1.synchronize()
        ms_e = e0.elapsed_time(e1) / steps
        res[T] = {"ms_per_step_replay": round(ms, 3), "frames_per_s_replay": round(B * T / ms * 1e3, 1),
                  "ms_per_step_eager": round(ms_e, 3), "tokens": int(model.last_num_tokens),
                  "loss": round(float(loss.item()), 5)}
        print(f"T={T}: replay {ms:.3f} ms/step ({B * T / ms * 1e3:,.0f} frames/s), eager {ms_e:.3f} ms/step, "
              f"N={model.last_num_tokens}", flush=True)
    # rotation: a different shape every step (the padded-batch pattern), all replays
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    frames = 0
    for i in range(3 * steps):
        T = Ts[i % 3]
        step(*data[T])
        frames += B * T
    e1.record()
    e1.synchronize()
    ms_rot = e0.elapsed_time(e1) / (3 * steps)
    out = {"what": "GraphedTrainStep, default HybridViT bf16 train step (fwd + CombinedLoss + bwd + clip + AdamW), "
                   f"B={B} x [1, 257, T], T rotating over {Ts}",
           "per_shape": res, "rotation_ms_per_step": round(ms_rot, 3),
           "rotation_frames_per_s": round(frames / (ms_rot * 3 * steps) * 1e3, 1),
           "captures": step.captures, "replays": step.replays, "cached": len(step.cache)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
