"""Data-parallel gradient exchange (dp.py) on CPU: world_size 2 over gloo.

The HybridViT DP step shards the batch across ranks and
all-reduces gradients once per step.  These tests check, on a small stand-in
module with the same parameter kinds (a pos_embed table whose gradient lives
only in its first N rows, a parameter used twice, an unused parameter), that
the bucketed hook-driven reducer yields exactly the full-batch mean gradient
on every rank, and that broadcast_module aligns parameters and buffers.
"""

import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class SlotLinear(torch.autograd.Function):
    """x @ w^T whose weight gradient is written straight into the reducer's
    bucket slot when one is published (functional.grad_dest), as the HIP
    linear / conv weight-gradient launches do: .grad then aliases the flat
    buffer that the bucket all-reduce sums in place."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, g):
        import hvit_amd.functional as HF

        x, w = ctx.saved_tensors
        dw = g.reshape(-1, g.shape[-1]).t() @ x.reshape(-1, x.shape[-1])
        dest = HF.grad_dest(id(w), tuple(w.shape))
        if dest is not None:
            dest.copy_(dw)
            dw = dest
        return g @ w, dw


class SlotFc(torch.nn.Linear):
    def forward(self, x):
        return SlotLinear.apply(x, self.weight) + self.bias


class Toy(torch.nn.Module):
    """Stand-in with HybridViT's gradient shapes of interest (fc1's weight
    gradient lands in its bucket slot like the HIP weight gradients)."""

    def __init__(self):
        super().__init__()
        self.pos_embed = torch.nn.Parameter(torch.randn(1, 50, 8) * 0.1)
        self.fc1 = SlotFc(8, 32)
        self.fc2 = torch.nn.Linear(32, 8)
        self.shared = torch.nn.Parameter(torch.randn(8) * 0.1)
        self.unused = torch.nn.Parameter(torch.zeros(3))
        self.register_buffer("running", torch.zeros(8))

    def forward(self, x):  # x [B, N, 8], N <= 50
        n = x.shape[1]
        self.last_num_tokens = n
        self.running.add_(1.0)  # a per-replica buffer update (like BN running stats)
        h = x + self.pos_embed[:, :n]
        h = h * self.shared
        h = self.fc2(torch.nn.functional.gelu(self.fc1(h)))
        return (h + self.shared).pow(2).mean()


def _worker(rank, world, port, bucket_mb, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import importlib

        import hvit_amd_loader

        hvit_amd_loader.load()
        dp = importlib.import_module("hvit_amd.dp")
        torch.manual_seed(100 + rank)  # ranks start different: broadcast must fix it
        model = Toy()
        model.running.fill_(float(rank + 1))
        dp.broadcast_module(model)
        torch.manual_seed(7)
        x = torch.randn(4 * world, 12, 8)
        n_tok = x.shape[1]
        red = dp.GradAllReducer(model, bucket_mb=bucket_mb, sliced={"pos_embed": n_tok})
        for step in range(2):  # two steps: reducer state must reset between them
            model.zero_grad(set_to_none=True)
            xs = x[rank * 4:(rank + 1) * 4] * (step + 1)
            model(xs).backward()
            red.finish()
        # full-batch reference: mean over ranks of the per-shard grads
        ref = Toy()
        ref.load_state_dict(model.state_dict())
        grads = {n: torch.zeros_like(p) for n, p in ref.named_parameters()}
        for r in range(world):
            ref.zero_grad(set_to_none=True)
            ref(x[r * 4:(r + 1) * 4] * 2).backward()
            for n, p in ref.named_parameters():
                if p.grad is not None:
                    grads[n] += p.grad / world
        import hvit_amd.functional as HF

        # the slot path was taken: fc1's .grad is a view of its bucket buffer
        adopted = any(model.fc1.weight.grad.data_ptr() == f.data_ptr() + 0 or
                      f.data_ptr() <= model.fc1.weight.grad.data_ptr() < f.data_ptr() + 4 * f.numel()
                      for fl in red.flats for f in fl if f is not None)
        assert HF.GRAD_DEST, "no bucket slots published"
        err = 0.0 if adopted else 1.0
        for n, p in model.named_parameters():
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            err = max(err, (g - grads[n]).abs().max().item())
        tail = model.pos_embed.grad[:, n_tok:].abs().max().item()
        q.put((rank, err, tail, model.running[0].item(), model.fc1.weight.sum().item(), len(red.buckets)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb", [25.0, 0.0005])
def test_grad_allreduce_matches_full_batch(bucket_mb):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    for rank, err, tail, running, wsum, nb in out:
        assert err < 1e-6, (rank, err)
        assert tail == 0.0
        assert running == 3.0  # rank 0's buffers (1, then +1 per forward) broadcast by finish()
    assert out[0][4] == out[1][4]  # identical parameters after broadcast
    if bucket_mb < 0.01:
        assert out[0][5] > 1  # several buckets exercised


def _worker_accum(rank, world, port, mode, q):
    """Gradient accumulation (trainer.py:164-183): two micro-batches per step,
    with hooks live on both (mode 'hooks': buckets already reduced in place --
    fc1's weight gradient lives in the bucket buffer -- are turned into means
    before the second micro-batch accumulates, then re-reduced) or the
    first under no_sync() (mode 'no_sync'); zero_grad with set_to_none False
    (grads stay views of the reducer's buffers) or True."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import importlib

        import hvit_amd_loader

        hvit_amd_loader.load()
        dp = importlib.import_module("hvit_amd.dp")
        torch.manual_seed(3)
        model = Toy()
        dp.broadcast_module(model)
        torch.manual_seed(9)
        xs = [torch.randn(4 * world, 12, 8) for _ in range(6)]
        red = dp.GradAllReducer(model, bucket_mb=0.0005, sliced={"pos_embed": 16})
        to_none = mode.endswith("none")
        errs = []
        for step in range(3):
            model.zero_grad(set_to_none=to_none)
            a, b = xs[2 * step], xs[2 * step + 1]
            if mode.startswith("no_sync"):
                with red.no_sync():
                    model(a[rank * 4:(rank + 1) * 4]).backward()
            else:
                model(a[rank * 4:(rank + 1) * 4]).backward()
            model(b[rank * 4:(rank + 1) * 4]).backward()
            red.finish()
            ref = Toy()
            ref.load_state_dict(model.state_dict())
            grads = {n: torch.zeros_like(p) for n, p in ref.named_parameters()}
            for r in range(world):
                for xx in (a, b):
                    ref.zero_grad(set_to_none=True)
                    ref(xx[r * 4:(r + 1) * 4]).backward()
                    for n, p in ref.named_parameters():
                        if p.grad is not None:
                            grads[n] += p.grad / world
            errs.append(max(((p.grad if p.grad is not None else torch.zeros_like(p)) - grads[n]).abs().max().item()
                            for n, p in model.named_parameters()))
        # token bound: a forward with more tokens than the sliced rows raises
        raised = False
        model.zero_grad(set_to_none=True)
        model(torch.randn(4, 20, 8)).backward()
        try:
            red.finish()
        except RuntimeError:
            raised = True
        # only rank 0 exceeds the bound: the ranks agree on the maximum first,
        # so EVERY rank raises (none is left waiting in a bucket collective)
        raised_one = False
        model.zero_grad(set_to_none=True)
        model(torch.randn(4, 20 if rank == 0 else 10, 8)).backward()
        try:
            red.finish()
        except RuntimeError:
            raised_one = True
        # and the reducer still works afterwards
        model.zero_grad(set_to_none=True)
        model(torch.randn(4, 10, 8)).backward()
        red.finish()
        q.put((rank, max(errs), raised and raised_one))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["hooks_none", "hooks_keep", "no_sync_none", "no_sync_keep"])
def test_grad_accumulation(mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_accum, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, err, raised in out:
        assert err < 1e-6, (mode, rank, err)
        assert raised


def _worker_subgroup(rank, world, port, q):
    """A GradAllReducer on a subgroup, built by that subgroup's ranks only: its
    host (gloo) group for the token-bound agreement is created with local
    synchronization (a plain new_group would wait for the ranks outside it);
    and GraphedTrainStep's per-call agreement takes the MIN of the ranks' flags."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import importlib
        import types

        import hvit_amd_loader

        hvit_amd_loader.load()
        dp = importlib.import_module("hvit_amd.dp")
        ts = importlib.import_module("hvit_amd.train_step")
        sub = dist.new_group([0, 1])  # (every rank takes part in creating the subgroup itself)
        ok_sub = True
        if rank < 2:
            real = dist.get_backend
            dist.get_backend = lambda g=None: "nccl"  # the reducer's data group as RCCL: it needs a gloo host group
            try:
                torch.manual_seed(3)
                model = Toy()
                red = dp.GradAllReducer(model, bucket_mb=0.0005, group=sub, sliced={"pos_embed": 16})
                red2 = dp.GradAllReducer(model, bucket_mb=0.0005, group=sub, sliced={"pos_embed": 16})
                ok_sub = red._host_group is red2._host_group and red._host_group is not sub
            finally:
                dist.get_backend = real
            red2.remove()
            model.zero_grad(set_to_none=True)
            model(torch.randn(4, 12, 8) * (rank + 1)).backward()
            red.finish()  # the token agreement runs on the locally created gloo group
            ok_sub = ok_sub and model.fc1.weight.grad is not None
            red.remove()
        # GraphedTrainStep's path agreement (gloo MIN over the reducer's host group)
        fake = types.SimpleNamespace(_agree=True, _host_group=None, world=world)
        g = ts.GraphedTrainStep(None, None, types.SimpleNamespace(capturable=True), reducer=fake)
        agree = (g._every_rank(rank != 1), g._every_rank(True), g._every_rank(False))
        # uniform_shapes: the caller's promise replaces the agreement (no collective)
        gu = ts.GraphedTrainStep(None, None, types.SimpleNamespace(capturable=True), reducer=fake,
                                 uniform_shapes=True)
        ok_sub = ok_sub and gu._every_rank(rank != 1) == (rank != 1)
        dist.barrier()
        q.put((rank, ok_sub, agree))
    finally:
        dist.destroy_process_group()


def test_subgroup_host_group_and_path_agreement():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_subgroup, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_sub, agree in out:
        assert ok_sub, rank
        assert agree == (False, True, False), (rank, agree)
