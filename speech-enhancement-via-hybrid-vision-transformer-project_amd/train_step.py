"""A whole training step captured in a hipGraph per input shape (SURVEY §8(f)
rank 3: variable-length batches).

The reference trainer steps through batches whose time axis varies from batch
to batch: ``collate_fn`` right-pads T to the batch maximum
(data/dataset.py:297-347), so a VoiceBank epoch sees many [B, 1, 257, T]
shapes, and ``Trainer.train_epoch`` runs forward, loss, backward, clip and the
optimizer on each (training/trainer.py:142-183).  Replaying one captured graph
needs one static shape, so ``GraphedTrainStep`` keeps one graph per input
shape (LRU-capped):

* the first ``warmup`` steps of a new shape run eagerly (they are real steps:
  they allocate the step's memory, build the bf16 weight shadows and optimizer
  state, and agree the data-parallel token bound); the next step of that shape
  is captured -- capture executes nothing -- and replayed, and every later
  step of that shape is a replay: the batch is copied into the graph's static
  input buffers first;
* every replay is a full, distinct step: the model draws its dropout seeds
  from a device-side counter and FusedAdamW(capturable=True) keeps its step
  counters on the device, so a replayed step equals the eager step it stands
  for (the train step is deterministic: bit for bit, tests/test_gpu_graph_cache.py);
* each graph has its own memory pool; evicting the least recently used graph
  (``max_graphs``) frees its pool;
* the optimizer's hyper-parameters are read on the device
  (``FusedAdamW.sync_hyper`` before every call), so a replay uses the current
  learning rate of an LR scheduler (trainer.py:304-309), not the captured one;
* under data parallelism (a ``GradAllReducer`` over more than one rank) every
  call first agrees over a gloo group whether any rank must run an eager step;
  then all ranks do, so no rank waits in a collective (RCCL on the eager group,
  or a sliced reducer's host agreement) that a replaying rank never enters.

``step(noisy, clean)`` returns the loss as a device tensor (the graph's static
output for replays: read it before the next call with the same shape).
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Callable, Optional

import torch

from . import functional as HF


class _Entry:
    __slots__ = ("seen", "graph", "x", "t", "loss")

    def __init__(self):
        self.seen = 0
        self.graph = None
        self.x = self.t = self.loss = None


class GraphedTrainStep:
    """forward + ``loss_fn`` + backward [+ ``reducer.finish()``] +
    ``optimizer.step()`` + ``zero_grad(set_to_none=True)``, replayed from a
    per-shape hipGraph after ``warmup`` eager steps of that shape."""

    def __init__(self, model: torch.nn.Module, loss_fn: Callable, optimizer, reducer=None, max_graphs: int = 8,
                 warmup: int = 2, uniform_shapes: bool = False):
        if getattr(optimizer, "capturable", True) is False:
            raise ValueError("hvit GraphedTrainStep: the optimizer must keep its step counters on the device "
                             "(FusedAdamW(..., capturable=True))")
        if max_graphs < 1 or warmup < 1:
            raise ValueError("hvit GraphedTrainStep: max_graphs and warmup must be >= 1")
        self.model, self.loss_fn, self.opt, self.reducer = model, loss_fn, optimizer, reducer
        self.max_graphs, self.warmup = max_graphs, warmup
        # the caller guarantees every rank sees the same sequence of input shapes
        # (e.g. a length-bucketing sampler shared by the ranks): every rank's mode
        # is then the same by construction and the per-call agreement is skipped
        self.uniform_shapes = uniform_shapes
        self.cache: "OrderedDict[tuple, _Entry]" = OrderedDict()
        self.captures = 0
        self.replays = 0
        self.eager_steps = 0
        self._side: Optional[torch.cuda.Stream] = None

    def _eager(self, x, t):
        loss = self.loss_fn(self.model(x), t)
        loss.backward()
        if self.reducer is not None:
            self.reducer.finish()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        # the step is done: hand back the value only, so a caller holding it does not
        # keep this step's AccumulateGrad nodes (side stream) alive into a capture
        return loss.detach()

    @staticmethod
    def _key(x, t):
        return (tuple(x.shape), x.dtype, tuple(t.shape), t.dtype, x.device)

    def _every_rank(self, flag: bool) -> bool:
        """True when ``flag`` holds on every rank of the reducer's group.  Ranks
        must agree on eager vs replay: a replayed step's bucket all-reduces run on
        the reducer's capture group (dp.capture_group) and an eager step's on its
        own group, so a rank replaying while another runs eager would wait in
        collectives of different communicators (and a sliced reducer's eager
        finish() also runs a host gloo agreement a replay never enters).  So every
        call agrees first -- one gloo all-reduce of a flag, outside any graph --
        and all ranks run eager when any of them must.  Cost: host time only (one
        8-byte gloo all-reduce, measured 0.22 / 0.49 / 0.86 ms at 2 / 4 / 8 ranks
        on an 8-CPU host), which overlaps the previous replay's GPU time (~5 ms);
        ``uniform_shapes=True`` skips it when the caller feeds every rank the same
        shape sequence (every rank's mode is then the same by construction)."""
        r = self.reducer
        if r is None or getattr(r, "world", 1) <= 1 or self.uniform_shapes:
            return flag
        import torch.distributed as dist

        t = torch.tensor([1 if flag else 0], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=r._host_group)
        return bool(t[0])

    def __call__(self, noisy: torch.Tensor, clean: torch.Tensor) -> torch.Tensor:
        key = self._key(noisy, clean)
        e = self.cache.get(key)
        if e is None:
            e = self.cache[key] = _Entry()
            while len(self.cache) > self.max_graphs:
                self.cache.popitem(last=False)  # the graph and its pool go with the entry
        self.cache.move_to_end(key)
        # the optimizer's device hyper-parameters follow param_groups (an LR
        # scheduler may have changed them since the graph was captured)
        sync = getattr(self.opt, "sync_hyper", None)
        if sync is not None:
            sync()
        mode = "replay" if e.graph is not None else ("eager" if e.seen < self.warmup else "capture")
        if not self._every_rank(mode != "eager"):
            mode = "eager"
        if mode == "replay":
            e.x.copy_(noisy)
            e.t.copy_(clean)
            # the replay updates the parameters without version bumps: drop the
            # inference forwards' packed / BN-folded weight copies
            HF.prep_cache_clear()
            e.graph.replay()
            self.replays += 1
            return e.loss
        if mode == "eager":
            # eager steps of a new shape (on a side stream, as capture warm-ups must be,
            # so the allocations they leave are not tied to the capture stream)
            if e.graph is None:
                e.seen += 1
            if self._side is None:
                self._side = torch.cuda.Stream(device=noisy.device)
            side = self._side
            side.wait_stream(torch.cuda.current_stream(noisy.device))
            with torch.cuda.stream(side):
                loss = self._eager(noisy, clean)
            torch.cuda.current_stream(noisy.device).wait_stream(side)
            self.eager_steps += 1
            return loss
        # capture (executes nothing), then replay it as this call's step
        e.x = noisy.detach().clone()
        e.t = clean.detach().clone()
        if self.reducer is not None:
            from .dp import quiesce_for_capture
            quiesce_for_capture(noisy.device)  # (captured collectives go to dp.capture_group)
        else:
            torch.cuda.synchronize(noisy.device)
        g = torch.cuda.CUDAGraph()
        # thread-local capture: a data-parallel reducer's process-group watchdog
        # thread polls earlier collectives' events, which a global-mode capture
        # would count as an illegal call and abort on
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            e.loss = self._eager(e.x, e.t)
        # the replays' loss buffer without the captured autograd graph (whose
        # AccumulateGrad nodes would outlive the capture and meet later eager
        # steps on another stream)
        e.loss = e.loss.detach()
        e.graph = g
        self.captures += 1
        g.replay()
        self.replays += 1
        return e.loss
