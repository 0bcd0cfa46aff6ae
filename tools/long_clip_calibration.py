"""Calibration evidence for tests/test_gpu_model.py::test_long_clip_bf16_vs_oracle
(verdict r4, item 7).

The default HybridViT on one ~4 s clip [1, 1, 256, 496] (496 tokens: the
chunked N > 256 attention forward and the KMAX = 512 backward), dropout-free
bf16 train step.  For every parameter gradient it records the relative L2
error against the fp32 CPU oracle of (a) this build and (b) torch bf16
autocast of the same oracle -- the calibration the test's bar (ours <= 2 x
autocast + 1e-2) rests on -- for BOTH inputs the test has used:

  * "rand":        torch.rand(1, 1, 256, 496) from Generator seed 11 (the
                   round-4 input on which the qkv weight gradient measured
                   1.25e-1 against a fixed 5e-2 bar);
  * "spectrogram": oracle/closed_form.spectrogram seeds 81 / 82 (the input the
                   test uses since round 4).

Writes a JSON line and a table (per parameter group: the worst ours / autocast
pair and the worst ratio) to stdout and to gpurun_out/long_clip_calibration.*

    python tools/long_clip_calibration.py
"""

import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hvit_amd_loader  # noqa: E402
from oracle import closed_form as CF  # noqa: E402
from oracle import hvit_oracle as O  # noqa: E402


def relnorm(a, b):
    a = torch.as_tensor(np.asarray(a)).double()
    b = torch.as_tensor(np.asarray(b)).double()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def run(hv, x, t):
    cfg = O.HViTConfig()
    cfg.dropout = cfg.attn_dropout = cfg.drop_path_rate = 0.0
    shapes = O.state_dict_shapes(cfg)
    W = CF.weights(shapes)
    m = hv.HybridViT(**cfg.as_kwargs(), precision="bf16").cuda()
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    sd = O.make_state(shapes, W, requires_grad=True)
    lo = O.combined_loss(O.forward(sd, x, cfg, training=True), t)
    lo.backward()
    sdg = {k: v.detach().cuda().requires_grad_(v.requires_grad) for k, v in sd.items()}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        yb = O.forward(sdg, x.cuda(), cfg, training=True)
    lb = O.combined_loss(yb.float(), t.cuda())
    lb.backward()
    loss = hv.CombinedLoss()(m.train()(x.cuda()), t.cuda())
    loss.backward()
    torch.cuda.synchronize()
    rows = []
    for k, p in m.named_parameters():
        got, ref, tb = p.grad.detach().cpu(), sd[k].grad, sdg[k].grad.detach().float().cpu()
        if k == "pos_encoding.pos_embed":
            got, ref, tb = got[:, :496], ref[:, :496], tb[:, :496]
        rows.append((k, relnorm(got, ref), relnorm(tb, ref)))
    return {"loss_ours": loss.item(), "loss_autocast": lb.item(), "loss_oracle": lo.item(), "rows": rows}


def main():
    hv = hvit_amd_loader.load()
    g = torch.Generator().manual_seed(11)
    xr = torch.rand(1, 1, 256, 496, generator=g)
    tr = torch.rand(1, 1, 256, 496, generator=g)
    xs = torch.as_tensor(CF.spectrogram((1, 1, 256, 496), 81))
    ts = torch.as_tensor(CF.spectrogram((1, 1, 256, 496), 82))
    out, lines = {}, []
    for name, (x, t) in {"rand": (xr, tr), "spectrogram": (xs, ts)}.items():
        r = run(hv, x, t)
        groups = {}
        for k, e, et in r["rows"]:
            grp = ".".join(k.split(".")[:2]) if k.startswith("transformer.blocks") else k.split(".")[0]
            w = groups.setdefault(grp, {"worst_ours": (0.0, 0.0, ""), "worst_ratio": (0.0, 0.0, 0.0, "")})
            if e > w["worst_ours"][0]:
                w["worst_ours"] = (e, et, k)
            ratio = e / max(et, 1e-12)
            if ratio > w["worst_ratio"][0]:
                w["worst_ratio"] = (ratio, e, et, k)
        qkv = [(k, e, et) for k, e, et in r["rows"] if k.endswith("attn.qkv.weight")]
        worst_qkv = max(qkv, key=lambda z: z[1])
        passes = all(e <= 2 * et + 1e-2 for _, e, et in r["rows"])
        out[name] = {"loss": (r["loss_ours"], r["loss_autocast"], r["loss_oracle"]), "groups": groups,
                     "worst_qkv_weight": worst_qkv, "all_within_2x_autocast_plus_1e-2": passes,
                     "rows": [(k, round(e, 5), round(et, 5)) for k, e, et in r["rows"]]}
        lines.append(f"== input {name}: loss ours {r['loss_ours']:.6f}  autocast {r['loss_autocast']:.6f}  "
                     f"oracle {r['loss_oracle']:.6f};  every gradient within 2 x autocast + 1e-2: {passes}")
        lines.append(f"   worst qkv weight gradient: {worst_qkv[0]}  ours {worst_qkv[1]:.3e}  autocast {worst_qkv[2]:.3e}")
        lines.append(f"   {'group':28s} {'worst ours':>11s} {'(autocast)':>11s}   {'worst ours/autocast':>20s}  parameter")
        for grp, w in groups.items():
            e, et, k = w["worst_ours"]
            ra, e2, et2, k2 = w["worst_ratio"]
            lines.append(f"   {grp:28s} {e:11.3e} {et:11.3e}   {ra:8.2f} ({e2:.2e}/{et2:.2e})  {k2}")
    text = "\n".join(lines)
    print(text, flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "long_clip_calibration.txt"), "w") as f:
        f.write(text + "\n")
    with open(os.path.join(ROOT, "gpurun_out", "long_clip_calibration.json"), "w") as f:
        json.dump(out, f)
    print(json.dumps({k: {"worst_qkv_weight": v["worst_qkv_weight"], "ok": v["all_within_2x_autocast_plus_1e-2"]}
                      for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
