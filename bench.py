"""HybridViT training-step throughput on MI355X (BASELINE.json metric).

One step = one HybridViT forward (train mode, dropout on) + CombinedLoss +
backward + [DP gradient all-reduce] + clip_grad_norm_(1.0) + AdamW step (the
clip fused into hvit FusedAdamW), at
batch 32 per GPU of 1x256x256 synthetic magnitude spectrograms, bf16 compute
(f32 master weights / statistics / gradients).  A frame is one STFT column, so
one spectrogram = 256 frames.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Rank 0 prints one JSON line.  After the timed steps, an instrumented repeat
of the same steps records HIP events around every launch of each op class
(functional.timed) on the stream it runs on; ``op_table`` lists each class's
GPU time per step and algorithmic FLOP/s (or bytes/s) against its roofline,
and ``roofline`` is the class with the most GPU time (the ViT linear
weight-gradient GEMMs at the default config; ``traffic`` from the committed
PMC pass, profiles/roofline_pmc.json).  ``cpu_baseline`` times the CPU
oracle (oracle/, fp32 PyTorch restatement of the reference) on a bounded
sample of the same step, on this host's cores.
"""

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FRAMES = 256
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--graph", type=int, default=None, choices=[0, 1],
                    help="1: capture one whole step (fwd + loss + bwd + clip + AdamW, device-side dropout seeds and "
                         "AdamW step counters; under DP also the hook-launched bucket all-reduces and the "
                         "reducer's finish) in a hipGraph and replay it; 0: eager launches.  Default 1")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 32; 16 for --variant large)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--mode", default="train", choices=["train", "infer"],
                    help="infer: BASELINE config 2 (forward only, eval, no grad)")
    ap.add_argument("--variant", default="default", choices=["default", "large"],
                    help="large: BASELINE config 5 shape (D=768, 12 heads, 12 layers)")
    ap.add_argument("--attn", default="bf16", choices=["bf16", "fp8"],
                    help="fp8: e4m3 MFMA attention forward (BASELINE config 5), bf16 attention backward")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the dominant op class, re-run in isolation (rocprofv3 --pmc passes)")
    ap.add_argument("--roofline-op", default="vit_linear_wgrad",
                    help="op class for --roofline-only (functional.timed tag with a recorded replay)")
    a = ap.parse_args()
    if a.graph is None:
        a.graph = 1
    if a.batch is None:
        a.batch = 16 if a.variant == "large" else 32
    return a


PEAKS = {"mfma": (PEAK_BF16_TFLOPS, "TFLOP/s", 1e12), "hbm": (PEAK_HBM_GBS, "GB/s", 1e9)}
# op class (functional.timed tag) -> roofline that bounds it
OP_BOUND = {"vit_linear_wgrad": "mfma", "vit_linear_fwd": "mfma", "vit_linear_dgrad": "mfma", "linear_wgrad": "mfma",
            "attn_fwd": "mfma", "attn_bwd": "mfma", "conv_fwd": "mfma", "conv_dgrad": "mfma", "conv_wgrad": "mfma",
            "bn_act_fwd": "hbm", "bn_act_bwd": "hbm", "layernorm_fwd": "hbm", "layernorm_bwd": "hbm",
            "dropout_scale": "hbm", "adamw": "hbm", "c1block_stats": "hbm", "c1block_fwd": "hbm", "c1block_bwd": "hbm"}
# "abi:<entry>" classes (functional._abi_timer: every other C-ABI call, no work figure) are "hbm" rows
# with time and launches only, so the table covers the whole step


def op_table(times, steps):
    """Per op class: launches and GPU ms per step, algorithmic work / time vs
    its roofline (HIP event pairs recorded on the launch stream in-step)."""
    rows = {}
    for name, recs in times.items():
        t = sum(e0.elapsed_time(e1) for e0, e1, _ in recs) / 1e3  # s
        known = all(w is not None for _, _, w in recs)
        work = sum(w for _, _, w in recs) if known else None
        bound = OP_BOUND.get(name, "hbm" if name.startswith("abi:") else "mfma")
        peak, unit, scale = PEAKS[bound]
        ach = work / t / scale if (known and t > 0) else None
        rows[name] = {"bound": bound, "ms_per_step": round(t / steps * 1e3, 4), "launches_per_step": len(recs) // steps,
                      "avg_launch_us": round(t / len(recs) * 1e6, 2),
                      "achieved": round(ach, 2) if ach is not None else None, "peak": peak, "unit": unit,
                      "frac": round(ach / peak, 4) if ach is not None else None,
                      "work_per_launch": work / len(recs) if known else None}
    return dict(sorted(rows.items(), key=lambda kv: -kv[1]["ms_per_step"]))


def roofline_of(table):
    """The dominant op class (most GPU time per step, among those with an
    algorithmic work figure) in the roofline format."""
    name, r = next((k, v) for k, v in table.items() if v["achieved"] is not None)
    return {"kernel": name, "bound": r["bound"], "achieved": r["achieved"], "peak": r["peak"], "unit": r["unit"],
            "frac": r["frac"], "traffic": measured_traffic(name), "avg_launch_us": r["avg_launch_us"],
            "launches_per_step": r["launches_per_step"],
            ("flops_per_launch" if r["bound"] == "mfma" else "bytes_per_launch"): r["work_per_launch"],
            "measured": "HIP events around each launch of this op class on its stream, inside an instrumented "
                        "repeat of the timed steps"}


def roofline_graph(step, name, reps=10):
    """The launches of op class ``name`` recorded from one real step
    (functional.REPLAY), captured ``reps`` times in one hipGraph and replayed
    between two HIP events: the class's average launch duration as the graph-
    replayed step runs it, with no per-launch event pair in the window (the
    instrumented repeat's events around each eager launch add their dispatch)
    -- what the rocprofv3 kernel statistics of the same command report for the
    class's kernels.  Returns (us per launch, work per launch) or None."""
    HF = sys.modules["hvit_amd.functional"]
    HF.REPLAY = {}
    try:
        step()
    finally:
        rec, HF.REPLAY = HF.REPLAY, None
    ops = rec.get(name)
    if not ops:
        return None
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # (warm-up off the default stream, as a capture wants)
        for fn, _ in ops:
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):  # (the recorded launches issue on the current stream: the capture stream)
        for _ in range(reps):
            for fn, _ in ops:
                fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / (reps * len(ops)))
    del g
    return sorted(ts)[1], sum(w for _, w in ops) / len(ops)


def roofline_loop(step, name=None, reps=20):
    """Re-run the launches of one op class, recorded from one real train step
    (functional.REPLAY), ``reps`` times on the same tensors: the dominant op in
    isolation for rocprofv3 --kernel-trace / --pmc passes (bench.py
    --roofline-only), timed with HIP events on its stream like the in-step
    table.  ``name`` None = the weight-gradient class with the most work."""
    HF = sys.modules["hvit_amd.functional"]
    HF.REPLAY = {}
    step()
    rec, HF.REPLAY = HF.REPLAY, None
    if name is None or name not in rec:
        name = max(rec, key=lambda k: sum(w for _, w in rec[k]))
    ops = rec[name]
    for fn, _ in ops:
        fn()
    torch.cuda.synchronize()
    HF.OP_TIMES = {}
    for _ in range(reps):
        for fn, w in ops:
            with HF.timed(name, w):
                fn()
    torch.cuda.synchronize()
    t = op_table(HF.OP_TIMES, reps)
    HF.OP_TIMES = None
    return roofline_of(t)


WORKLOAD = {"variant": "default", "mode": "train", "batch": 32}  # this run's (set in main)


def measured_traffic(name):
    """HBM bytes per launch of op class ``name`` from the committed PMC pass
    (profiles/roofline_pmc.json, written from rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes over ``bench.py --roofline-only``; FETCH_SIZE doubled per
    the gfx950 correction).  None when absent or recorded for another op or
    another workload (the pass is of the default B=32 train step)."""
    p = os.path.join(ROOT, "profiles", "roofline_pmc.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    if not all(d.get(k, v) == v for k, v in WORKLOAD.items()):
        return None
    if "ops" in d:  # several op classes, one PMC pair each (tools/roofline_pmc.py)
        return d["ops"].get(name, {}).get("hbm_bytes_per_launch")
    return d.get("hbm_bytes_per_launch") if d.get("op") == name else None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(batch, budget_s):
    """Oracle (fp32 PyTorch CPU restatement of the reference) train step:
    fwd + CombinedLoss + bwd + clip + AdamW on the same synthetic
    spectrograms, bounded by ``budget_s``."""
    from hvit_amd.data import spectrogram_batch
    from oracle import closed_form as CF
    from oracle import hvit_oracle as O

    # every core this process may run on, capped by OMP_NUM_THREADS when the
    # host sets it (the GPU box's CPU share: its affinity mask can name the whole machine)
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    if os.environ.get("OMP_NUM_THREADS", "").isdigit() and int(os.environ["OMP_NUM_THREADS"]) > 0:
        cores = min(cores, int(os.environ["OMP_NUM_THREADS"]))
    if os.environ.get("HVIT_CPU_THREADS"):
        cores = int(os.environ["HVIT_CPU_THREADS"])
    torch.set_num_threads(cores)
    cfg = O.HViTConfig()
    shapes = O.state_dict_shapes(cfg)
    sd = O.make_state(shapes, CF.weights(shapes), requires_grad=True)
    params = [v for k, v in sd.items() if v.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-4, weight_decay=0.01)
    x, t = spectrogram_batch(batch, seed=1234)

    def step():
        y = O.forward(sd, x, cfg, training=True)
        loss = O.combined_loss(y, t)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    t1 = time.perf_counter()
    step()  # warmup
    print(f"cpu baseline: warmup step {time.perf_counter() - t1:.1f} s on {cores} threads", file=sys.stderr, flush=True)
    times = []
    t0 = time.perf_counter()
    while len(times) < 3 and (time.perf_counter() - t0) < budget_s:
        t1 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t1)
        print(f"cpu baseline: step {len(times)} {times[-1]:.1f} s", file=sys.stderr, flush=True)
    times.sort()
    dt = times[len(times) // 2]
    # the B=32 eval forward too (BASELINE config 2's CPU counterpart; the survey's
    # 1.82 s reference figure is this measurement): 1 warmup + best of 2
    with torch.no_grad():
        O.forward(sd, x, cfg, training=False)
        fts = []
        for _ in range(2):
            t1 = time.perf_counter()
            O.forward(sd, x, cfg, training=False)
            fts.append(time.perf_counter() - t1)
    ft = min(fts)
    print(f"cpu baseline: eval forward {ft:.2f} s", file=sys.stderr, flush=True)
    return {"value": round(batch * FRAMES / dt, 2), "unit": "spectrogram-frames/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu": cpu_model(),
            "sample": f"oracle/hvit_oracle.py fp32 train step (fwd+CombinedLoss+bwd+clip+AdamW), B={batch}, "
                      f"1x256x256 synthetic spectrograms, 1 warmup + {len(times)} timed steps, median "
                      f"{dt:.2f} s/step (all: {', '.join(f'{t:.2f}' for t in times)})",
            "fwd_value": round(batch * FRAMES / ft, 2),
            "fwd_sample": f"the same oracle's B={batch} eval forward (no grad), 1 warmup + best of 2: {ft:.2f} s"}


def main():
    args = parse()
    WORKLOAD.update(variant=args.variant, mode=args.mode, batch=args.batch)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HVIT_FORCE_DIST=1: the DP branch (process group + GradAllReducer) even at
    # world size 1 -- exercises the RCCL path on a one-GPU box
    use_dist = world > 1 or os.environ.get("HVIT_FORCE_DIST") == "1"
    if use_dist:
        # one process per GPU over RCCL; HVIT_DIST_BACKEND=gloo (with ranks sharing the
        # visible GPUs round-robin) only rehearses the DP path on a one-GPU box
        backend = os.environ.get("HVIT_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group(backend)
    import hvit_amd_loader

    hv = hvit_amd_loader.load()
    from hvit_amd.data import spectrogram_batch
    from hvit_amd.dp import GradAllReducer, broadcast_module

    torch.manual_seed(1234)
    arch = dict(embed_dim=768, num_heads=12, num_layers=12) if args.variant == "large" else {}
    model = hv.HybridViT(precision=args.precision, attention_precision="fp8" if args.attn == "fp8" else None,
                         **arch).cuda().train()
    reducer = None
    if use_dist:
        broadcast_module(model)
        reducer = GradAllReducer(model, bucket_mb=25, sliced={"pos_encoding.pos_embed": FRAMES})
    # AdamW (training/optimizer.py:53-61) with clip_grad_norm_(1.0) (trainer.py:170-174) fused into it;
    # capturable: device step counters, so the captured step replays with the right bias corrections
    opt = hv.FusedAdamW(model.parameters(), lr=1e-4, weight_decay=0.01, max_grad_norm=1.0,
                        capturable=bool(args.graph))
    crit = hv.CombinedLoss()
    noisy, clean = spectrogram_batch(args.batch, seed=1234 + rank * args.batch)
    noisy, clean = noisy.cuda(), clean.cuda()
    torch.manual_seed(1000 + rank)

    if args.mode == "infer":
        model.eval()

    def step():
        if args.mode == "infer":
            with torch.no_grad():
                return model(noisy).float().mean()
        y = model(noisy)
        loss = crit(y, clean)
        loss.backward()
        if reducer is not None:
            reducer.finish()
        opt.step()  # clip to 1.0 + AdamW
        opt.zero_grad(set_to_none=True)
        return loss

    if args.roofline_only:
        for _ in range(2):
            step()
        print(json.dumps(roofline_loop(step, args.roofline_op)), flush=True)
        return
    eager_step = step
    graph = None
    if args.graph:
        # warm up eagerly on a side stream (allocator pools, weight shadows,
        # optimizer state, device step counters, both generations of the DP
        # bucket buffers, the token-bound agreement), then capture one whole
        # step; every replay is a full step: new dropout masks (device seed
        # stream), AdamW bias corrections from the device step counters, and
        # under DP the bucket all-reduces over RCCL (captured from the hooks
        # in backward order, then the reducer's wait + average)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(2, args.warmup // 2)):
                step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if use_dist:
            from hvit_amd.dp import quiesce_for_capture
            quiesce_for_capture()  # device idle; the captured collectives go to dp.capture_group
        graph = torch.cuda.CUDAGraph()
        # thread-local capture: under DP the process group's watchdog thread
        # polls the events of earlier collectives; in the default (global) mode
        # that poll during the capture invalidates it (hipErrorStreamCaptureUnsupported)
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            static_loss = step()
        # keep the replays' loss buffer but not the captured autograd graph: its
        # AccumulateGrad nodes (created on the capture stream) would otherwise stay
        # alive and be reused by the eager repeats below on another stream (torch's
        # "AccumulateGrad node's stream does not match" warning, and a cross-stream
        # sync in those eager steps; the captured graph itself is unaffected)
        static_loss = static_loss.detach()

        def step():
            graph.replay()
            return static_loss
    for _ in range(args.warmup):
        step()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    # per-step HIP events on the stream (no host sync inside the timed region)
    # give the median step; the wall clock around all K steps gives the mean
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        loss = step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_step = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    ms_median = per_step[len(per_step) // 2]
    if use_dist:
        te = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed = te.item()
    ms = elapsed / args.steps * 1e3
    spectros = world * args.batch * args.steps / elapsed
    value = spectros * FRAMES
    if not torch.isfinite(loss).item():
        raise RuntimeError("non-finite loss")

    # host enqueue cost of one step while the GPU queue is busy (no sync inside)
    HF = sys.modules["hvit_amd.functional"]
    step()
    t1 = time.perf_counter()
    for _ in range(3):
        step()
    host_ms = (time.perf_counter() - t1) / 3 * 1e3
    torch.cuda.synchronize()
    eager_ms = None
    if graph is not None:
        # the same step launched eagerly (for the record: host-launch bound or not)
        for _ in range(2):
            eager_step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(5):
            eager_step()
        torch.cuda.synchronize()
        eager_ms = (time.perf_counter() - t1) / 5 * 1e3
    # instrumented repeat of the timed steps (eager: HIP events around every
    # launch of each op class, functional.timed) for the per-op roofline table
    isteps = min(args.steps, 10)
    # each instrumented step is queued behind a GPU spin of ~1.5 eager steps, so
    # the host enqueues the whole step while the GPU is busy and no host
    # launch gap falls inside an op's event window (the eager host enqueue is
    # slower than the GPU step: unqueued, its gaps inflated the classes with the
    # most host work per launch)
    spin = None
    if hasattr(torch.cuda, "_sleep"):
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1 << 20)
        c0.record()
        torch.cuda._sleep(1 << 22)
        c1.record()
        c1.synchronize()
        per_ms = (1 << 22) / max(c0.elapsed_time(c1), 1e-3)
        spin = min(int(per_ms * 1.5 * max(eager_ms or 0.0, ms * 1.5, 5.0)), 1 << 28)
    HF.OP_TIMES = {}
    for _ in range(isteps):
        if spin:
            torch.cuda._sleep(spin)
        eager_step()
    torch.cuda.synchronize()
    table = op_table(HF.OP_TIMES, isteps)
    HF.OP_TIMES = None

    out = None
    roof = roofline_of(table) if rank == 0 else None
    if world == 1 and roof is not None:
        # the dominant class re-timed as a graph replay of its recorded launches (no per-launch events)
        try:
            gr = roofline_graph(eager_step, roof["kernel"])
        except RuntimeError as exc:  # (the per-launch event figure stands; the line says why)
            gr = None
            roof["graph_timing_error"] = str(exc)[:200]
        if gr is not None:
            us, work = gr
            _, _, scale = PEAKS[roof["bound"]]
            ach = work / (us * 1e-6) / scale
            roof.update({"event_avg_launch_us": roof["avg_launch_us"], "event_frac": roof["frac"],
                         "avg_launch_us": round(us, 2), "achieved": round(ach, 2),
                         "frac": round(ach / roof["peak"], 4),
                         "measured": "HIP events around a hipGraph replay of this op class's launches recorded "
                                     "from one real step (10 repetitions; no per-launch events -- the instrumented "
                                     "repeat's per-launch event figure in event_avg_launch_us / event_frac)"})
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.mode == "train" and args.variant == "default":
            cpu = cpu_baseline(args.batch, args.cpu_seconds)
        out = {
            "metric": ("spectrogram-frames/sec/GPU (fwd+bwd) on 256x256 mag-spec, batch 32; 1/2/4/8 GPU"
                       if args.mode == "train" else "spectrogram-frames/sec/GPU (fwd only, eval) on 256x256 mag-spec"),
            "value": round(value, 1),
            "unit": "spectrogram-frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "ms_per_step_median": round(ms_median, 3),
            "launch": "hipGraph replay of the whole step" if graph is not None else "eager",
            "ms_per_step_eager": round(eager_ms, 3) if eager_ms is not None else round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision + ("+fp8-attention" if args.attn == "fp8" else ""),
            "data": "synthetic (harmonic+noise 16 kHz waveforms, host STFT 512/128 hann, min-max, 256x256)",
            "config": {"workload": (("HybridViT default (enc 64/128/256, 6x8-head d512 ViT, dec 256/128/64/1)"
                                     if args.variant == "default" else
                                     "HybridViT large (enc 64/128/256, 12x12-head d768 ViT, dec 256/128/64/1)")
                                    + (" train step: fwd + CombinedLoss + bwd + clip + AdamW" if args.mode == "train"
                                       else " inference forward (eval, no grad)")),
                       "global_batch": world * args.batch, "seq_len": 256, "input": [args.batch, 1, 256, 256],
                       "parallelism": f"dp{world}",
                       "dist_backend": dist.get_backend() if use_dist else None},
            "spectrograms_per_s": round(spectros, 2),
            "frames_per_s_per_gpu": round(value / world, 1),
            "value_is": "aggregate spectrogram frames/s over all n_gpus (per-GPU figure: frames_per_s_per_gpu)",
            "host_enqueue_ms_per_step": round(host_ms, 3),
            "host_enqueue_is": "graph replay call" if graph is not None else "eager launches of one step",
            "final_loss": round(loss.item(), 6),
            "roofline": roof,
            "op_table": {k: {kk: vv for kk, vv in v.items() if kk != "work_per_launch"} for k, v in table.items()},
            "op_table_sum_ms_per_step": round(sum(v["ms_per_step"] for v in table.values()), 3),
            "op_table_is": "eager instrumented repeat: HIP events around every op class and every other C-ABI call "
                           "('abi:' rows); the sum covers the whole step's kernels",
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
