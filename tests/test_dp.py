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


class Toy(torch.nn.Module):
    """Stand-in with HybridViT's gradient shapes of interest."""

    def __init__(self):
        super().__init__()
        self.pos_embed = torch.nn.Parameter(torch.randn(1, 50, 8) * 0.1)
        self.fc1 = torch.nn.Linear(8, 32)
        self.fc2 = torch.nn.Linear(32, 8)
        self.shared = torch.nn.Parameter(torch.randn(8) * 0.1)
        self.unused = torch.nn.Parameter(torch.zeros(3))
        self.register_buffer("running", torch.zeros(8))

    def forward(self, x):  # x [B, N, 8], N <= 50
        n = x.shape[1]
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
        err = 0.0
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
        assert running == 1.0  # buffers broadcast from rank 0
    assert out[0][4] == out[1][4]  # identical parameters after broadcast
    if bucket_mb < 0.01:
        assert out[0][5] > 1  # several buckets exercised
