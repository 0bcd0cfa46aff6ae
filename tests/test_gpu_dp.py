"""GPU: the data-parallel HybridViT step (BASELINE config 4) with
the real HIP model on every rank.  Two ranks share cuda:0 over gloo (RCCL
refuses two ranks on one device; the 8-GPU RCCL run is the driver's).  Each
rank runs the tiny HybridViT (fp32, dropout off, train-mode BN = local BN per
replica) on its batch shard under GradAllReducer; the reduced gradients must
equal the mean of the per-shard gradients computed single-process, replicas
must stay bit-identical through FusedAdamW steps, and rank 0's BN statistics
must be broadcast.  The input has N = 260 > 256 patch tokens, so pos_embed rows
beyond 256 carry gradient (reduced through ``sliced`` rows = 320)."""

import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KW = dict(encoder_channels=[8, 16, 32], embed_dim=64, num_heads=4, num_layers=2, decoder_channels=[32, 16, 8, 1],
          dropout=0.0, attn_dropout=0.0, drop_path_rate=0.0, precision="fp32")
SHAPE = (2, 1, 64, 1040)   # per rank; N = (64/16) * (1040/16) = 4 * 65 = 260 tokens


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import copy
        import importlib

        import hvit_amd_loader

        hv = hvit_amd_loader.load()
        dp = importlib.import_module("hvit_amd.dp")
        torch.cuda.set_device(0)
        torch.manual_seed(11 + rank)  # ranks start different: broadcast_module aligns them
        model = hv.HybridViT(**KW).cuda().train()
        dp.broadcast_module(model)
        ref = copy.deepcopy(model)
        g = torch.Generator().manual_seed(5)
        x = torch.rand((world * SHAPE[0],) + SHAPE[1:], generator=g)
        t = torch.rand(x.shape, generator=g)
        crit = hv.CombinedLoss()
        red = dp.GradAllReducer(model, bucket_mb=0.05, sliced={"pos_encoding.pos_embed": 320})
        sl = slice(rank * SHAPE[0], (rank + 1) * SHAPE[0])
        crit(model(x[sl].cuda()), t[sl].cuda()).backward()
        # the ViT and conv weight gradients were written into their bucket slots
        # (functional.GRAD_DEST): .grad already lives in the flat buffer
        def in_bucket(p):
            flat = red.flats[red.where[id(p)]][red._gen]
            return p.grad.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()
        adopted = all(in_bucket(p) for p in (model.transformer.blocks[0].attn.qkv.weight,
                                             model.transformer.blocks[-1].mlp.net[3].weight,
                                             model.encoder[1].block[0].weight))
        red.finish()
        ntok = model.last_num_tokens
        # single-process reference: mean of the per-shard gradients (local BN per shard)
        acc = {n: torch.zeros_like(p) for n, p in ref.named_parameters()}
        for r in range(world):
            m = copy.deepcopy(ref)
            s2 = slice(r * SHAPE[0], (r + 1) * SHAPE[0])
            crit(m(x[s2].cuda()), t[s2].cuda()).backward()
            for n, p in m.named_parameters():
                acc[n] += p.grad / world
        err = max(((p.grad - acc[n]).norm() / acc[n].norm().clamp_min(1e-20)).item()
                  for n, p in model.named_parameters())
        pos_tail = model.pos_encoding.pos_embed.grad[0, 256:ntok].abs().max().item()
        beyond = model.pos_encoding.pos_embed.grad[0, ntok:].abs().max().item()
        bn = model.encoder[0].bn.running_mean.clone()
        bn0 = bn.clone()
        dist.broadcast(bn0, 0)
        # replicas stay identical through optimizer steps
        opt = hv.FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        for _ in range(2):
            crit(model(x[sl].cuda()), t[sl].cuda()).backward()
            red.finish()
            opt.step()
            opt.zero_grad(set_to_none=True)
        # plain floats: a tensor in the queue is shared by file descriptor, which
        # the parent can only open while this process is still alive
        csum = torch.stack([p.detach().double().sum() for p in model.parameters()]).cpu().tolist()
        q.put((rank, err, pos_tail, beyond, ntok, torch.equal(bn, bn0), csum, adopted))
    finally:
        dist.destroy_process_group()


def test_dp_hybridvit_two_ranks_on_one_gpu():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, pos_tail, beyond, ntok, bn_same, _, adopted in out:
        assert adopted             # weight gradients written in place in the bucket (no launch copy)
        assert ntok == 260
        assert err < 1e-5, (rank, err)
        assert pos_tail > 0.0      # rows 256..259 carry gradient and were reduced
        assert beyond == 0.0
        assert bn_same             # rank 0's running statistics on every rank
    assert out[0][6] == out[1][6]  # bit-identical replicas after 3 optimizer steps


def test_rccl_world1_bench_dp_branch():
    """BASELINE config 4's code path on RCCL: bench.py's DP branch
    (init_process_group("nccl", device_id=cuda:0), broadcast_module,
    GradAllReducer over RCCL every step, FusedAdamW) launched through
    torch.distributed.run at world size 1 on the box's one GPU
    (HVIT_FORCE_DIST=1).  The 8-GPU scaling run is the driver's."""
    import json
    import subprocess

    env = dict(os.environ, HVIT_FORCE_DIST="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--steps", "3",
           "--warmup", "1", "--batch", "4", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    # (the first error lines name the failing call; the tail holds the launcher's report)
    errs = [ln for ln in r.stderr.splitlines() if "rror" in ln or "what()" in ln or "fault" in ln.lower()][:20]
    assert r.returncode == 0, "\n".join(errs) + "\n...\n" + r.stderr[-2500:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["config"]["dist_backend"] == "nccl"
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "dp1"
    # the DP step is captured whole (bucket all-reduces from the hooks included)
    assert out["launch"] == "hipGraph replay of the whole step"
    assert out["value"] > 0 and abs(out["final_loss"]) < 1e3
    # one grouped weight-gradient launch per step: the DP buckets wait for it instead of splitting it
    assert out["op_table"]["vit_linear_wgrad"]["launches_per_step"] == 1, out["op_table"]["vit_linear_wgrad"]


def test_rccl_world1_dp_graph_matches_eager():
    """The captured DP step (RCCL, world 1: hook-launched bucket all-reduces,
    finish(), FusedAdamW capturable, dropout on) replays exactly the steps an
    eager copy takes from the same dropout seed state: parameters equal after
    each of 3 replays (bitwise: the train step is deterministic), losses equal,
    step counters advanced on the device."""
    import json
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dp_graph_worker.py"), str(_free_port())],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["dropout_state_equal"]
    # the buckets holding ViT weights wait for the one grouped weight-gradient launch (not one launch per bucket)
    assert out["group_launches_per_step"] == 1.0, out
    assert out["steps"] == 5.0  # 2 warm-up + 3 replays
    for a, b in out["losses"]:
        assert abs(a - b) <= 1e-6 * abs(b), out["losses"]
    assert out["exact"], out["rel"]


def test_rccl_world1_graph_cache_matches_eager():
    """Verdict r4 item 8: GraphedTrainStep WITH a GradAllReducer over RCCL (world
    1) on three input shapes, bit-identical to an eager DP copy after every step
    (tests/dp_graph_cache_worker.py)."""
    import json
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dp_graph_cache_worker.py"), str(_free_port())],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["bad"] == [], out
    assert out["dropout_state_equal"]
    assert out["captures"] >= 4 and out["replays"] >= 6 and out["cached"] <= 2, out


def _worker_accum(rank, world, port, q):
    """Two micro-batches per optimizer step with the hooks live on both and
    zero_grad(set_to_none=True) (trainer.py:164-183 under DP): the ViT and conv
    weight gradients of the first micro-batch live in the bucket buffers and are
    reduced there in place before the second backward accumulates."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import copy
        import importlib

        import hvit_amd_loader

        hv = hvit_amd_loader.load()
        dp = importlib.import_module("hvit_amd.dp")
        torch.cuda.set_device(0)
        torch.manual_seed(11)
        kw = dict(KW)
        model = hv.HybridViT(**kw).cuda().train()
        ref = copy.deepcopy(model)
        g = torch.Generator().manual_seed(6)
        xs = [torch.rand((world * 2, 1, 64, 64), generator=g) for _ in range(2)]
        ts = [torch.rand((world * 2, 1, 64, 64), generator=g) for _ in range(2)]
        crit = hv.CombinedLoss()
        red = dp.GradAllReducer(model, bucket_mb=0.05)
        sl = slice(rank * 2, (rank + 1) * 2)
        model.zero_grad(set_to_none=True)
        for x, t in zip(xs, ts):
            crit(model(x[sl].cuda()), t[sl].cuda()).backward()
        red.finish()
        acc = {n: torch.zeros_like(p) for n, p in ref.named_parameters()}
        for r in range(world):
            m = copy.deepcopy(ref)
            s2 = slice(r * 2, (r + 1) * 2)
            for x, t in zip(xs, ts):
                crit(m(x[s2].cuda()), t[s2].cuda()).backward()
            for n, p in m.named_parameters():
                acc[n] += p.grad / world
        err = max(((p.grad - acc[n]).norm() / acc[n].norm().clamp_min(1e-20)).item()
                  for n, p in model.named_parameters())
        q.put((rank, err))
    finally:
        dist.destroy_process_group()


def test_dp_accumulation_hooks_set_to_none_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_accum, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err in out:
        assert err < 1e-5, (rank, err)
