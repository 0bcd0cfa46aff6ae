"""Data-parallel gradient averaging for the HybridViT training step.

The reference has no distributed code; the build adds the one
exchange the path has: the gradient all-reduce of a batch-sharded step.  One
process per GPU, ``torch.distributed`` with the RCCL backend ("nccl" on ROCm)
over xGMI; gloo works for CPU tests and for ranks that share one GPU.

* Gradients are bucketed (default 25 MB) in reverse registration order, which
  is roughly the order backward produces them.  A bucket's all-reduce is
  launched from a post-accumulate-grad hook as soon as its last gradient lands,
  so communication overlaps the rest of the backward.
* Every bucket owns two persistent flat buffers used on alternate steps.  The
  next step's buffer is published before its backward (functional.GRAD_DEST):
  the ViT linear and conv weight-gradient launches write their result straight
  into the parameter's slot, autograd adopts that view as ``.grad`` and the
  bucket launch finds it in place (no copy).  Other gradients (biases, norms,
  and any gradient accumulated onto an existing ``.grad``) are copied into the
  buffer at the launch.  After the reduction each ``.grad`` is a view of the
  averaged buffer: no concatenation buffer and no copy-back.  Alternating keeps
  a launch from ever reducing in place under a ``.grad`` view that a later
  accumulating backward still writes (``zero_grad(set_to_none=False)``).
* Gradient accumulation (trainer.py:72, :164-183: several backward passes
  before one optimizer step) is exact.  A bucket is reduced in place (its
  ``.grad`` views ARE the flat buffer), so when a later backward brings a
  gradient for a bucket whose all-reduce was already launched, a pre-accumulate
  hook first waits for that reduction and divides the buffer by the world size:
  the views then hold mean(g1) on every rank, the backward adds its local g2,
  and the bucket is reduced again (mean over ranks of mean(g1) + g2 =
  mean(g1 + g2)).  ``no_sync()`` skips the wasted early launches.
* Capturable: a whole DP step (forward, backward with the hook-launched bucket
  all-reduces, ``finish()``, the optimizer) can be captured in one hipGraph and
  replayed; nothing in the hooks or in ``finish()`` syncs the host with the
  device.
* ``sliced={"pos_encoding.pos_embed": R}`` reduces only the first R rows of a
  parameter whose gradient is zero beyond the token count (the 10 000-row
  positional table; 18 % of the default model's gradient bytes at N = 256).
  R must bound the token count of every forward on every rank; the model's
  ``last_num_tokens`` is agreed over the group (MAX) in ``finish()`` on a gloo
  group (host memory: no device sync) and a larger count raises on every rank.
  Under stream capture the agreement is skipped: a captured step replays the
  shapes of the eager warm-up steps that were checked.  Without ``sliced`` the
  whole table is reduced (exact for any N).
* BatchNorm statistics are computed per replica (local BN, as DDP without
  SyncBN; the reference has no distributed code to match).  With
  ``broadcast_buffers`` (default, as DDP) rank 0's running statistics are
  broadcast to every rank (one coalesced broadcast launched when a training
  forward ends, overlapped with the backward, installed in ``finish()``), so
  replicas never diverge and any rank's ``state_dict`` equals rank 0's.
* Buckets close at 25 MB and, once past 4 MB, where the top-level component
  changes, so the last bucket (the exposed tail of the step) is the encoder's
  1.5 MB rather than a mix with the first ViT block's gradients.
"""

from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import weakref

import torch
import torch.distributed as dist

from . import functional as HF

# Captured collectives run on a process group of their own.  Round 5 saw the
# process group's watchdog thread abort a DP step capture (RCCL, world 1:
# "operation not permitted on an event last recorded in a capturing stream").
# The watchdog polls the end event of every collective issued OUTSIDE a capture
# (hipEventQuery on ProcessGroupNCCL's work list, ~every 100 ms, until it sees
# the event complete); those events are recorded on the group's internal NCCL
# stream.  A collective issued during a capture on the SAME group makes that
# stream join the capture, and HIP refuses a query of an event whose recording
# stream is capturing -- so any eager bucket all-reduce the watchdog had not yet
# retired when the capture began killed the process.  Now every collective a
# capture contains goes to a second NCCL group (``capture_group``) whose
# communicator is connected eagerly (ncclCommSplit / eager_connect: no
# collective) and which never runs a collective outside a capture; captured
# collectives are never put on the watchdog's list (ProcessGroupNCCL enqueues
# only uncaptured works).  So the watchdog's list holds only the eager group's
# works, whose stream never joins a capture: no poll can meet a capturing
# stream, whatever the timing.  (Round 5's stopgap slept 0.35 s before every
# capture; gone.)
_GROUPS: Dict[tuple, tuple] = {}


def _cached_group(kind: str, group, make):
    """One helper group per (default group, kind, ranks): the entry keeps the
    default group OBJECT it was made under and is reused only while that same
    object is the default group (a destroy_process_group() + re-init gives a new
    one, possibly at the same id())."""
    ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(dist.get_world_size()))
    key = (kind, ranks)
    e = _GROUPS.get(key)
    if e is not None and e[0] is dist.group.WORLD:
        return e[1]
    g = make(ranks)
    _GROUPS[key] = (dist.group.WORLD, g)
    return g


def _gloo_group(group):
    """A gloo group over ``group``'s ranks, reused (set_rows() rebuilds the
    reducer).  Created with local synchronization, so only the member ranks take
    part: a reducer built on a subgroup by that subgroup's ranks alone does not
    wait for the others."""
    return _cached_group("gloo", group, lambda ranks: dist.new_group(ranks=list(ranks), backend="gloo",
                                                                     use_local_synchronization=True))


def capture_group(group=None):
    """The NCCL group that carries a reducer's collectives while a hipGraph is
    being captured (see above).  Its communicator is connected here, without a
    collective.  On the world group every rank calls this (the reducer is built
    on every rank); a subgroup's is made by its members alone, which a default
    group bound to a device (ncclCommSplit from the parent) does not allow."""
    def make(ranks):
        sub = group is not None and len(ranks) != dist.get_world_size()
        bound = getattr(dist.distributed_c10d._get_default_group(), "bound_device_id", None) is not None
        if sub and bound:
            return None  # (capture with such a reducer raises in GradAllReducer._coll_group)
        g = dist.new_group(ranks=list(ranks), backend="nccl", use_local_synchronization=sub)
        dev = torch.device("cuda", torch.cuda.current_device())
        be = g._get_backend(dev)
        if hasattr(be, "eager_connect_single_device"):
            be.eager_connect_single_device(dev)  # (idempotent when new_group already split it)
        return g

    return _cached_group("capture", group, make)


def quiesce_for_capture(device=None) -> None:
    """Call right before capturing a step that contains collectives: the
    device is idle (the eager warm-up's collectives have finished).  No wait
    for the watchdog is needed (see capture_group)."""
    torch.cuda.synchronize(device)


class GradAllReducer:
    def __init__(self, model: torch.nn.Module, bucket_mb: float = 25.0, group=None,
                 sliced: Optional[Dict[str, int]] = None, broadcast_buffers: bool = True):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)
        self.sliced = dict(sliced or {})
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        self.params = [p for _, p in named]
        self.names = {id(p): n for n, p in named}
        for n in self.sliced:
            if n not in dict(named):
                raise KeyError(f"hvit GradAllReducer: no parameter {n!r} to slice")
        self.bucket_mb = bucket_mb
        cap = int(bucket_mb * 1024 * 1024)
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size, top = [], 0, None
        for n, p in reversed(named):
            nbytes = self._numel(p) * 4
            # a bucket of at least 4 MB also closes where the top-level component
            # changes: the last bucket launched is then the early encoder's few
            # weights alone, not a 25 MB mix with the first ViT block's, whose
            # gradients were ready long before (the last bucket's all-reduce is the
            # exposed tail of the step); smaller ones merge on (collective latency)
            t = n.split(".")[0]
            if cur and (size + nbytes > cap or (t != top and size >= (4 << 20))):
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
            top = t
        if cur:
            self.buckets.append(cur)
        self.where = {id(p): b for b, ps in enumerate(self.buckets) for p in ps}
        self.offsets = []
        for ps in self.buckets:
            offs, o = [], 0
            for p in ps:
                offs.append(o)
                o += self._numel(p)
            self.offsets.append((offs, o))
        self.flats: List[List[Optional[torch.Tensor]]] = [[None, None] for _ in self.buckets]
        self._gen = 0
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        # pre-accumulate hooks: a gradient arriving for an already-reduced bucket
        self._hooks += [p.register_hook(self._pre_grad_hook(p)) for p in self.params]
        self._bcast = []  # (work, flat, buffers) of the buffer broadcasts launched by training forwards
        self._fwd_hook = model.register_forward_hook(self._on_forward)
        self._syncing = True
        self.broadcast_buffers = broadcast_buffers
        self._max_tokens = 0
        # host-side group for the token-bound agreement: a CPU all_reduce on gloo
        # needs no device sync (on an nccl group an int read back would stall the
        # host until the whole backward had run)
        # (also GraphedTrainStep's per-call eager / replay agreement: a replaying rank's
        # collectives go to the capture group, an eager rank's to this group)
        self._agree = bool(self.sliced) and self.world > 1
        self._host_group = self.group
        if self.world > 1 and dist.get_backend(self.group) != "gloo":
            self._host_group = _gloo_group(self.group)
        # collectives issued inside a hipGraph capture go to their own NCCL group
        # (capture_group: the watchdog never polls a work of it)
        self._nccl = dist.get_backend(self.group) == "nccl" and torch.cuda.is_available()
        self._cap_group = capture_group(self.group) if self._nccl else None
        self.reset()
        self._publish()

    def _publish(self):
        """Allocate this generation's flat buffers and announce each unsliced
        parameter's slot in them to the weight-gradient launches."""
        for b, ps in enumerate(self.buckets):
            offs, total = self.offsets[b]
            flat = self.flats[b][self._gen]
            if flat is None or flat.device != ps[0].device:
                flat = self.flats[b][self._gen] = torch.empty(total, dtype=torch.float32, device=ps[0].device)
            for p, o in zip(ps, offs):
                if self._rows(p) is None:
                    HF.GRAD_DEST[id(p)] = (weakref.ref(p), flat, o)

    # ------------------------------------------------------------ helpers --
    def _rows(self, p):
        return self.sliced.get(self.names[id(p)])

    def _numel(self, p):
        rows = self._rows(p)
        return p[:, :rows].numel() if rows is not None else p.numel()

    def _view(self, p):
        rows = self._rows(p)
        return p.grad[:, :rows] if rows is not None else p.grad

    def _on_forward(self, module, args, out):
        n = getattr(module, "last_num_tokens", None)
        if n is not None:
            self._max_tokens = max(self._max_tokens, int(n))
        if self.broadcast_buffers and self.world > 1 and module.training:
            # the running statistics are final for this step once the forward has
            # run (the backward does not touch them): broadcast them now, overlapped
            # with the whole backward, and install them in finish()
            bufs = self._float_buffers()
            if bufs:
                with torch.no_grad():
                    fb = torch.cat([t.reshape(-1).float() for t in bufs])
                    work = dist.broadcast(fb, self._bcast_src(), group=self._coll_group(), async_op=True)
                self._bcast.append((work, fb, bufs))
                if len(self._bcast) > 4:  # forwards without a finish() (no-grad passes in train mode): keep the last
                    self._bcast.pop(0)[0].wait()

    def _coll_group(self):
        """The group for a collective issued now: the capture group while the
        current stream is being captured, else the reducer's group."""
        if self._nccl and torch.cuda.is_current_stream_capturing():
            if self._cap_group is None:
                raise RuntimeError("hvit GradAllReducer: capturing collectives on a subgroup needs a default "
                                   "process group not bound to a device (init_process_group without device_id)")
            return self._cap_group
        return self.group

    def _float_buffers(self):
        # the module's current buffers (a .to() / .cuda() since construction replaces them)
        return [b for b in self.model.buffers() if b.is_floating_point()]

    def _bcast_src(self):
        # the group's rank 0 as a global rank
        return dist.get_global_rank(self.group, 0) if self.group is not None else 0

    def set_rows(self, name: str, rows: int):
        """Change a sliced parameter's row bound (bucket sizes follow)."""
        if name not in self.sliced:
            raise KeyError(name)
        self.remove()
        self.__init__(self.model, bucket_mb=self.bucket_mb, group=self.group, sliced={**self.sliced, name: rows},
                      broadcast_buffers=self.broadcast_buffers)

    def reset(self):
        self.seen = [set() for _ in self.buckets]
        self.works = [None] * len(self.buckets)
        self.stale = [False] * len(self.buckets)

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulation micro-steps: gradients accumulate locally, no bucket
        is launched (DDP's no_sync); the step after the context syncs."""
        prev, self._syncing = self._syncing, False
        try:
            yield
        finally:
            self._syncing = prev

    # ----------------------------------------------------------- the hooks --
    def _pre_grad_hook(self, p):
        ref = weakref.ref(p)

        def hook(grad):
            q = ref()
            if q is not None:
                self._before_accumulate(q)
            return None

        return hook

    def _before_accumulate(self, p):
        """A backward is about to add a gradient to ``p``.  If ``p``'s bucket was
        already launched this step, its buffer holds the in-place SUM over ranks
        of the earlier gradients, and the GRAD_DEST ``.grad`` views are that
        buffer: wait for it and divide by the world size, so the views hold the
        mean and the bucket can be reduced again after this backward (the
        reduction is linear).  Copied gradients (biases, norms, sliced rows)
        still hold their local sums, which the relaunch copies in afresh."""
        b = self.where[id(p)]
        w = self.works[b]
        if w is None:
            return
        w.wait()
        flat = self.flats[b][self._gen]
        flat.div_(self.world)  # (the copied gradients' regions are re-copied at the relaunch)
        self.works[b] = None
        self.stale[b] = False
        self.seen[b] = set()

    def _on_grad(self, p):
        if not self._syncing:
            return
        b = self.where[id(p)]
        if self.works[b] is not None:  # (unreachable: the pre-accumulate hook reset it)
            self.stale[b] = True
            return
        self.seen[b].add(id(p))
        if len(self.seen[b]) == len(self.buckets[b]):
            self._launch(b)

    def _launch(self, b):
        ps = self.buckets[b]
        offs, total = self.offsets[b]
        dev = ps[0].grad.device
        flat = self.flats[b][self._gen]
        if flat is None or flat.device != dev:
            flat = self.flats[b][self._gen] = torch.empty(total, dtype=torch.float32, device=dev)
        if dev.type == "cuda" and HF.wgrad_pending(dev):
            # weight gradients queued for the grouped launch (functional.wgrad_enqueue)
            # are not written yet: reduce this bucket right after that launch (one
            # launch for every block -- flushing here split it into one per bucket,
            # 0.34 -> 0.56 ms/step at world 1 -- and the patch-embedding backward
            # flushes, so these buckets still reduce under the encoder backward)
            HF.wgrad_after_flush(dev, lambda b=b: self._launch(b))
            return
        ctx = contextlib.nullcontext()
        if dev.type == "cuda" and HF.side_pending(dev):
            # weight gradients still in flight on the side stream (functional.on_side):
            # copy and reduce from there, after everything issued on both streams
            s = HF.side_stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            ctx = torch.cuda.stream(s)
        with ctx:
            # the gradients not already in the bucket (biases, norms, sliced rows, accumulated ones):
            # one multi-tensor copy instead of a copy launch per tensor (~85 per step at ~5 us each)
            dsts, srcs = [], []
            for p, o in zip(ps, offs):
                v = self._view(p)
                dst = flat[o:o + v.numel()].view_as(v)
                if dst.data_ptr() != v.data_ptr():
                    dsts.append(dst)
                    srcs.append(v)
            if dsts:
                torch._foreach_copy_(dsts, srcs)
            self.works[b] = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self._coll_group(), async_op=True)

    def finish(self):
        """Wait for every bucket (launching any whose hooks did not fire, e.g.
        unused parameters or a step taken under no_sync, and re-launching stale
        ones), install the averaged gradients, broadcast rank 0's buffers, and
        reset for the next step."""
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        if self.sliced:
            # agree on the largest token count over the group first, so that a
            # rank whose batch exceeds the row bound makes EVERY rank raise here,
            # before any of them enters the bucket collectives below (host memory
            # on a gloo group: no device sync; skipped under capture, whose
            # static shapes the eager warm-up steps already agreed on)
            mt = self._max_tokens
            if self._agree and not capturing:
                t = torch.tensor([mt], dtype=torch.int64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._host_group)
                mt = int(t[0])
            for name, rows in self.sliced.items():
                if mt > rows:
                    self._max_tokens = 0
                    self.reset()
                    raise RuntimeError(f"hvit GradAllReducer: a forward used {mt} tokens but only "
                                       f"{rows} rows of {name} are reduced; raise sliced[{name!r}]")
        if torch.cuda.is_available():
            for dev in {p.device for ps in self.buckets for p in ps if p.device.type == "cuda"}:
                HF.wgrad_flush(dev)  # (normally done: the backward's final callback; runs deferred buckets)
        for b, ps in enumerate(self.buckets):
            if self.works[b] is not None and not self.stale[b]:
                continue
            if self.works[b] is not None:
                self.works[b].wait()
            for p in ps:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            self._launch(b)
        for b, ps in enumerate(self.buckets):
            self.works[b].wait()
            flat = self.flats[b][self._gen].div_(self.world)
            offs, _ = self.offsets[b]
            for p, o in zip(ps, offs):
                if self._rows(p) is not None:
                    v = self._view(p)
                    v.copy_(flat[o:o + v.numel()].view_as(v))
                else:
                    p.grad = flat[o:o + p.numel()].view_as(p)
        # rank 0's buffers: the broadcast the last training forward launched, or
        # (no forward through the module this step) one issued now
        pending, self._bcast = self._bcast, []
        for work, _, _ in pending[:-1]:
            work.wait()
        bcast = pending[-1] if pending else None
        if bcast is None and self.broadcast_buffers and self.world > 1:
            bufs = self._float_buffers()
            if bufs:
                with torch.no_grad():
                    fb = torch.cat([t.reshape(-1).float() for t in bufs])
                    bcast = (dist.broadcast(fb, self._bcast_src(), group=self._coll_group(), async_op=True), fb,
                             bufs)
        if bcast is not None:
            work, fb, bufs = bcast
            work.wait()
            with torch.no_grad():
                views, o = [], 0
                for t in bufs:
                    views.append(fb[o:o + t.numel()].view_as(t))
                    o += t.numel()
                torch._foreach_copy_(bufs, views)  # (one multi-tensor launch)
        self._max_tokens = 0
        self._gen ^= 1
        self.reset()
        self._publish()

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._fwd_hook.remove()
        for p in self.params:
            e = HF.GRAD_DEST.get(id(p))
            if e is not None and e[0]() is p:
                del HF.GRAD_DEST[id(p)]


def broadcast_module(model: torch.nn.Module, src: int = 0, group=None):
    """Make every rank start from rank ``src``'s parameters and buffers."""
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src, group=group)


def save_on_rank0(obj, path: str, group=None) -> bool:
    """torch.save(obj, path) on rank 0 only (Trainer.save_checkpoint,
    trainer.py:350-380, under DP), then a barrier so no rank reads the file
    before it is complete.  Returns True on the rank that wrote."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if rank == 0:
        torch.save(obj, path)
    if dist.is_initialized():
        dist.barrier(group=group)
    return rank == 0
