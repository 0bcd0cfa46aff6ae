"""In-container validation of the CPU baseline (SURVEY §8(d),
BASELINE.md §2-3): the oracle restatement (oracle/hvit_oracle.py, fp32) timed
on the B=32 eval forward and the B=32 train step (fwd + CombinedLoss + bwd +
clip + AdamW) with every affinity core, best of 3 after one warmup -- the
protocol of the survey's reference measurements (1.82 s / 5.79 s on 8 vCPU,
8 threads) -- and compared with them.  Output: profiles/r3_cpu_baseline_check.txt."""
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import hvit_amd_loader  # noqa: E402

hvit_amd_loader.load()
from hvit_amd.data import spectrogram_batch  # noqa: E402
from oracle import closed_form as CF  # noqa: E402
from oracle import hvit_oracle as O  # noqa: E402

REF = {"fwd": 1.82, "step": 5.79}  # BASELINE.md §2 (reference, survey container, 8 threads)
# the reference's B=32 eval-forward time by aten op (share of CPU time)
REF_SHARES = {"aten::mkldnn_convolution": 38.0, "aten::addmm": 20.0, "aten::copy_": 11.0,
              "aten::max_pool2d_with_indices": 10.0, "aten::bmm": 5.0, "aten::native_batch_norm": 4.0}


def lscpu():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keep = ("Model name", "CPU(s):", "Thread(s) per core", "Core(s) per socket", "Socket(s)", "Flags")
        return "\n".join(l if not l.startswith("Flags") else l[:120] + " ..." for l in out.splitlines()
                         if l.strip().startswith(keep))
    except Exception as e:  # noqa: BLE001
        return f"lscpu unavailable: {e}"


def best3(fn):
    fn()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), ts


def main():
    cores = len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    cfg = O.HViTConfig()
    shapes = O.state_dict_shapes(cfg)
    x, t = spectrogram_batch(32, seed=1234)
    sd_eval = O.make_state(shapes, CF.weights(shapes))

    def fwd():
        with torch.no_grad():
            O.forward(sd_eval, x, cfg, training=False)

    sd = O.make_state(shapes, CF.weights(shapes), requires_grad=True)
    params = [v for v in sd.values() if v.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-4, weight_decay=0.01)

    def step():
        y = O.forward(sd, x, cfg, training=True)
        O.combined_loss(y, t).backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    f, fs = best3(fwd)
    s, ss = best3(step)
    # the oracle's own op mix on the same forward (torch.profiler self CPU time):
    # the same aten ops in the same shares as the reference's profile means the
    # restatement does the reference's work, and a time ratio is the host's
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        fwd()
    ka = {e.key: e.self_cpu_time_total for e in prof.key_averages()}
    tot = sum(ka.values())
    share_lines = ["", "forward self-CPU share by aten op: oracle (this host) vs reference (SURVEY §6)"]
    for k, ref in REF_SHARES.items():
        share_lines.append(f"  {k:34s} {100.0 * ka.get(k, 0.0) / tot:5.1f} %   reference {ref:4.1f} %")
    lines = [
        f"host: {platform.node()}  torch {torch.__version__}  threads {torch.get_num_threads()} "
        f"(affinity cores {cores})",
        lscpu(),
        "",
        "oracle/hvit_oracle.py fp32, default HybridViT, B=32 x 1x256x256 synthetic spectrograms "
        "(hvit_amd.data.spectrogram_batch), 1 warmup + best of 3",
        f"  eval forward : {f:6.2f} s  (runs {', '.join(f'{v:.2f}' for v in fs)})  reference 1.82 s  "
        f"ratio {f / REF['fwd']:.3f}",
        f"  train step   : {s:6.2f} s  (runs {', '.join(f'{v:.2f}' for v in ss)})  reference 5.79 s  "
        f"ratio {s / REF['step']:.3f}",
        f"  frames/s (train): {32 * 256 / s:8.1f}   reference {32 * 256 / REF['step']:8.1f}",
    ] + share_lines
    out = "\n".join(lines)
    print(out)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", sys.argv[1] if len(sys.argv) > 1 else "cpu_baseline_check.txt"),
              "w") as fh:
        fh.write(out + "\n")


if __name__ == "__main__":
    main()
