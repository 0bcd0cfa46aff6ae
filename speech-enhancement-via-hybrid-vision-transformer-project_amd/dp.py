"""Data-parallel gradient averaging for the HybridViT training step.

The reference has no distributed code; the build adds the one
exchange the path has: the gradient all-reduce of a batch-sharded step.  One
process per GPU, ``torch.distributed`` with the RCCL backend ("nccl" on ROCm)
over xGMI; gloo works for CPU tests.

Gradients are bucketed (default 25 MB) in reverse registration order, which is
roughly the order backward produces them; a bucket's all-reduce is launched
from a post-accumulate-grad hook as soon as its last gradient lands, so
communication overlaps the rest of the backward.  BatchNorm statistics stay
per replica (no SyncBN in the reference).  ``pos_encoding.pos_embed`` only has
non-zero gradient in its first N rows (N patches), so only that slice is
reduced: 18 % fewer bytes for the default model, bit-identical result.
"""

from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist


class GradAllReducer:
    def __init__(self, model: torch.nn.Module, bucket_mb: float = 25.0, group=None,
                 sliced: Optional[Dict[str, int]] = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.sliced = dict(sliced or {})
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        self.params = [p for _, p in named]
        self.names = {id(p): n for n, p in named}
        cap = int(bucket_mb * 1024 * 1024)
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for n, p in reversed(named):
            nbytes = self._numel(p) * 4
            if cur and size + nbytes > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)
        self.where = {id(p): b for b, ps in enumerate(self.buckets) for p in ps}
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self.reset()

    def _numel(self, p):
        rows = self.sliced.get(self.names[id(p)])
        return p[:, :rows].numel() if rows is not None else p.numel()

    def _view(self, p):
        rows = self.sliced.get(self.names[id(p)])
        g = p.grad
        return g[:, :rows] if rows is not None else g

    def set_rows(self, name: str, rows: int):
        self.sliced[name] = rows

    def reset(self):
        self.pending = [len(b) for b in self.buckets]
        self.works = [None] * len(self.buckets)
        self.flats = [None] * len(self.buckets)

    def _on_grad(self, p):
        b = self.where[id(p)]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self._launch(b)

    def _launch(self, b):
        flat = torch.cat([self._view(p).reshape(-1) for p in self.buckets[b]])
        self.flats[b] = flat
        self.works[b] = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self):
        """Wait for every bucket (launching any whose hooks did not fire, e.g.
        unused parameters), write averaged gradients back, reset for the next
        step."""
        for b, ps in enumerate(self.buckets):
            if self.works[b] is None:
                for p in ps:
                    if p.grad is None:
                        p.grad = torch.zeros_like(p)
                self._launch(b)
        for b, ps in enumerate(self.buckets):
            self.works[b].wait()
            flat = self.flats[b].div_(self.world)
            off = 0
            for p in ps:
                v = self._view(p)
                n = v.numel()
                v.copy_(flat[off:off + n].view_as(v))
                off += n
        self.reset()

    def remove(self):
        for h in self._hooks:
            h.remove()


def broadcast_module(model: torch.nn.Module, src: int = 0, group=None):
    """Make every rank start from rank ``src``'s parameters and buffers."""
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src, group=group)
