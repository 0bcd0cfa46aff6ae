"""Autograd functions that run the HybridViT hot path on libhvit.so.

Each Function covers one reference module (cited) and chains C-ABI calls;
PyTorch autograd only sequences them and sums gradients where a tensor has two
consumers (the U-Net skips).  Activations are NHWC in the compute dtype
``dt`` (f32 parity path or bf16 throughput path); the ViT residual stream,
LayerNorm statistics, BatchNorm statistics and all parameter gradients are f32.
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Optional

import ctypes as C
import weakref

import torch

from . import _lib as L
from ._lib import call, ptr, stream_ptr

F32, BF16 = L.F32, L.BF16


# ---------------------------------------------------------------------------
# In-step op timing (measurement only; off unless a caller installs a table).
# bench.py installs OP_TIMES = {} around its timed region: every instrumented
# op records a HIP event pair on the stream it launches on, so an op's GPU
# duration is measured inside the real training step.  Off, `timed` is a no-op.
OP_TIMES = None


_DEPTH = 0  # open _Timed contexts (an op class covers the ABI calls inside it)


class _Timed:
    __slots__ = ("name", "work", "e0")

    def __init__(self, name, work):
        self.name, self.work = name, work

    def __enter__(self):
        global _DEPTH
        _DEPTH += 1
        self.e0 = torch.cuda.Event(enable_timing=True)
        self.e0.record()

    def __exit__(self, *exc):
        global _DEPTH
        _DEPTH -= 1
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        OP_TIMES.setdefault(self.name, []).append((self.e0, e1, self.work))


def _abi_timer(name, fn):
    """Every C-ABI call outside an explicit op class gets its own class
    ("abi:<entry>", no algorithmic work figure) while OP_TIMES is installed, so
    the op table attributes the whole step."""
    if OP_TIMES is None or _DEPTH > 0:
        return fn()
    with _Timed("abi:" + name[5:] if name.startswith("hvit_") else "abi:" + name, None):
        return fn()


L.TIMER = _abi_timer


class _Untimed:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_UNTIMED = _Untimed()


def timed(name: str, work: float):
    """Context for one op launch sequence; ``work`` = algorithmic FLOPs or bytes."""
    return _UNTIMED if OP_TIMES is None else _Timed(name, work)


# Launch recorder (measurement only): bench.py installs REPLAY = {} for one
# step; the recorded ops (ViT linears, weight gradients) then also store a closure that re-issues the
# same launch on the same tensors, so the dominant op class can be re-run in
# isolation (bench.py --roofline-only, the rocprofv3 / PMC loop).
REPLAY = None


def _record(name, fn):
    if REPLAY is not None:
        REPLAY.setdefault(name, []).append(fn)


def _launch(name, work, fn, e=None, keep=()):
    """One timed, recorded launch of op class ``name`` (the ViT forward and
    data-gradient linears: re-runnable in isolation for the roofline loop).
    ``fn(e[, stream])`` issues it with epilogue ``e`` (on the launch's own
    stream unless one is given).  The recorded replay runs the same launch without the
    epilogue's side job (the carried slab sum belongs to the step, and its
    slabs and destination are freed after the backward) and holds ``keep`` (the
    tensors behind the epilogue's raw pointers, e.g. gelu'(h) and the bias-grad
    accumulator) so the replay never touches freed memory."""
    with timed(name, work):
        fn(e)
    if REPLAY is not None:
        er = None
        if e is not None:
            er = type(e).from_buffer_copy(e)
            er.side = L.SlabSum()
        # (the replay launches on the stream current at replay time: bench.py may capture it)
        _record(name, ((lambda er=er, keep=keep: fn(er, stream_ptr())), work))


def _empty(shape, dt, dev):
    return torch.empty(shape, dtype=L.torch_dtype(dt), device=dev)


class ZSlot:
    """A zeroed f32 accumulator (atomic target) that one backward call needs:
    a slice of the forward pass's shared zero pool, or its own zeros when the
    pool was never flushed (a Function used outside HybridViT.forward)."""

    __slots__ = ("n", "t", "__weakref__")

    def __init__(self, n):
        self.n = n
        self.t = None

    def take(self, dev):
        t, self.t = self.t, None  # the caller's reference is the only one left
        return t if t is not None else torch.zeros(self.n, dtype=torch.float32, device=dev)


_ZPENDING = []


def zslot(n: int) -> ZSlot:
    """Register an accumulator for this forward's backward (see zflush)."""
    s = ZSlot(n)
    if len(_ZPENDING) > 4096:
        _ZPENDING[:] = [r for r in _ZPENDING if r() is not None]
    _ZPENDING.append(weakref.ref(s))
    return s


def zflush(dev) -> None:
    """Give every accumulator registered since the last flush its slice of ONE
    zeroed buffer: one fill per forward instead of a clear per backward call
    (LayerNorm dgamma/dbeta, BatchNorm slot sums, fused bias-grad column sums)."""
    live = [s for s in (r() for r in _ZPENDING) if s is not None and s.t is None]
    _ZPENDING.clear()
    if not live:
        return
    offs, tot = [], 0
    for s in live:
        offs.append(tot)
        tot += (s.n + 63) // 64 * 64  # 256-B aligned slices
    buf = torch.zeros(tot, dtype=torch.float32, device=dev)
    for s, o in zip(live, offs):
        s.t = buf[o:o + s.n]


def _zs(ctx, n):
    """zslot(n) when this Function's backward can run (an input needs grad)."""
    return zslot(n) if any(ctx.needs_input_grad) else None


# Cache of prepared weights, filled by prep_weights() with one multi-tensor
# launch: (id(param), kind, dt) -> (_sig(param), tensor, param, BN
# versions).  A lookup requires the parameter to be unmodified since
# preparation.  Entries survive from one forward to the next only for
# inference forwards (prep_weights(reuse=True): eval + no_grad, the caller
# drops the cache on every train()/eval() switch) -- a captured training step
# updates parameters without bumping their version counters, so training
# forwards always re-prepare.
_PREP = {}


def prep_cache_clear() -> None:
    _PREP.clear()


def _sig(t):
    """What a prepared copy of ``t`` is valid for: its version counter and its
    storage (``param.data = ...`` and ``.to()`` move the storage without a version
    bump; a replayed graph updates in place with neither, hence the clears in
    GraphedTrainStep and FusedAdamW.step)."""
    return (t._version, t.data_ptr())


def _prep_get(t, kind, dt):
    hit = _PREP.get((id(t), kind, dt))
    if hit is not None and hit[0] == _sig(t) and hit[2] is t:
        return hit[1]
    return None


def _bn_versions(bn):
    return tuple(_sig(x) for x in bn[:4]) + tuple(id(x) for x in bn[:4])


# Persistent bf16 copies of linear weights ("shadows"): id(param) ->
# [weakref(param), bf16 tensor, _sig(param) the copy matches or None].
# FusedAdamW writes a parameter's shadow in the same pass that updates the
# parameter (optim.py), so the next forward skips that cast.
_SHADOW = {}


def shadow_of(p):
    """The persistent bf16 shadow of ``p`` (None if ``p`` has none)."""
    e = _SHADOW.get(id(p))
    return e[1] if e is not None and e[0]() is p else None


def shadow_mark(p):
    """Record that ``p``'s shadow now equals bf16(p) at its current version."""
    e = _SHADOW.get(id(p))
    if e is not None and e[0]() is p:
        e[2] = _sig(p)


def prep_weights(items, dev, reuse: bool = False):
    """items: [(param, kind, dt)] or, kind 3, [(param, 3, dt, (gamma, beta,
    running_mean, running_var, eps))]; kind 0 = cast, 1/2 = conv pack mode 0/1,
    3 = mode-0 pack with eval BatchNorm folded in (prepared value: (packed
    weight, f32 bias)).  Replaces the cache with freshly prepared copies (one
    kernel launch); bf16 casts whose shadow is current are reused without a
    launch, and with ``reuse`` (inference forwards) so is every entry still
    current from the previous forward."""
    old = dict(_PREP) if reuse else {}
    _PREP.clear()
    todo = []
    for w, kind, dt, *bn in items:
        key = (id(w), kind, dt)
        hit = old.get(key)
        if (hit is not None and hit[2] is w and hit[0] == _sig(w) and
                (kind != 3 or hit[3] == _bn_versions(bn[0]))):
            _PREP[key] = hit  # unchanged since it was prepared (repeated inference forwards)
            continue
        if kind == 3:
            out = (_empty((w.numel(),), dt, dev), torch.empty(w.shape[0], dtype=torch.float32, device=dev))
            todo.append((w, kind, dt, out, bn[0]))
            continue
        if kind == 0 and L.dt_of(w) == dt:
            continue
        if kind == 0 and dt == BF16:
            e = _SHADOW.get(id(w))
            if e is None or e[0]() is not w or e[1].shape != w.shape:
                e = _SHADOW[id(w)] = [weakref.ref(w), _empty(w.shape, dt, dev), None]
            if e[2] == _sig(w):
                _PREP[(id(w), kind, dt)] = (_sig(w), e[1], w, None)
                continue
            todo.append((w, kind, dt, e[1], None))
            continue
        out = _empty(w.shape if kind == 0 else (w.numel(),), dt, dev)
        todo.append((w, kind, dt, out, None))
    if not todo:
        return
    arr = (L.WPrepItem * len(todo))()
    for i, (w, kind, dt, out, bn) in enumerate(todo):
        co, ci, ks = (w.shape[0], w.shape[1], w.shape[2]) if kind else (0, 0, 0)
        if kind == 3:
            gamma, beta, rmean, rvar, eps = bn
            arr[i] = L.WPrepItem(w.data_ptr(), out[0].data_ptr(), w.numel(), kind, dt, co, ci, ks, gamma.data_ptr(),
                                 beta.data_ptr(), rmean.data_ptr(), rvar.data_ptr(), out[1].data_ptr(), eps)
        else:
            arr[i] = L.WPrepItem(w.data_ptr(), out.data_ptr(), w.numel(), kind, dt, co, ci, ks)
    call("hvit_weight_prep", len(todo), arr, stream_ptr())
    for w, kind, dt, out, bn in todo:
        _PREP[(id(w), kind, dt)] = (_sig(w), out, w, _bn_versions(bn) if kind == 3 else None)
        if kind == 0 and dt == BF16:
            shadow_mark(w)


def cast(t: torch.Tensor, dt: int) -> torch.Tensor:
    """Contiguous copy of ``t`` in dtype ``dt`` (no copy if already there)."""
    hit = _prep_get(t, 0, dt)
    if hit is not None:
        return hit
    t = t.contiguous()
    if L.dt_of(t) == dt:
        return t
    out = _empty(t.shape, dt, t.device)
    call("hvit_cast", t.data_ptr(), L.dt_of(t), out.data_ptr(), dt, t.numel(), stream_ptr())
    return out


def pack_conv(w: torch.Tensor, mode: int, dt: int) -> torch.Tensor:
    hit = _prep_get(w, 1 + mode, dt)
    if hit is not None:
        return hit
    w = w.detach().contiguous()
    if w.dtype != torch.float32:
        raise TypeError("hvit: conv weights must be float32 parameters")
    co, ci, ks, _ = w.shape
    out = _empty((w.numel(),), dt, w.device)
    call("hvit_conv_weight_pack", w.data_ptr(), co, ci, ks, mode, out.data_ptr(), dt, stream_ptr())
    return out


# Data-parallel gradient slots (dp.GradAllReducer): id(param) -> (weakref(param),
# flat bucket buffer, offset).  A weight-gradient launch whose parameter has a
# slot (and no .grad yet) writes straight into it; autograd then adopts that
# view as .grad and the bucket's all-reduce copies nothing.
GRAD_DEST = {}


def grad_dest(pid, shape):
    """The bucket view for parameter ``pid``'s gradient, or None (no slot, or
    the parameter already holds a gradient that a second backward accumulates
    into)."""
    e = GRAD_DEST.get(pid)
    if e is None:
        return None
    ref, flat, o = e
    p = ref()
    n = math.prod(shape)
    if p is None or p.grad is not None or tuple(p.shape) != tuple(shape) or flat.numel() < o + n:
        return None
    return flat[o:o + n].view(shape)  # a fresh view each time: autograd can adopt it without a copy


def unpack_conv(dwp: torch.Tensor, shape, out=None) -> torch.Tensor:
    co, ci, ks, _ = shape
    dw = out if out is not None else torch.empty(shape, dtype=torch.float32, device=dwp.device)
    call("hvit_conv_weight_unpack", dwp.data_ptr(), co, ci, ks, dw.data_ptr(), stream_ptr())
    return dw


def col_sum(x: torch.Tensor, rows: int, cols: int) -> torch.Tensor:
    out = torch.empty(cols, dtype=torch.float32, device=x.device)
    call("hvit_reduce_rows", x.data_ptr(), L.dt_of(x), rows, cols, cols, 0, out.data_ptr(), stream_ptr())
    return out


def wgrad_tickets(M, N, K) -> int:
    """uint32 counters the in-kernel split-K reduction of linear_wgrad needs."""
    return int(L.lib().hvit_wgrad_tickets(M, N, K))


def linear_wgrad_deferred(dt, dy, x, M, N, K, tag="vit_linear_wgrad", dest=None, side: Optional[Deferred] = None):
    if not DEFER:  # A/B: the two-launch form (an incoming side job summed first)
        if side is not None:
            call("hvit_sum_slabs_strided", side.job.src, side.job.splits, side.job.stride, side.job.n, side.job.dst,
                 stream_ptr())
        return linear_wgrad(dt, dy, x, M, N, K, tag=tag, dest=dest), None
    """dw [N, K] = dy^T x (f32) with the split-K slab sum deferred: returns
    (dw, Deferred); dw is final once the Deferred has been passed as the side
    job of the next hvit_linear_fwd / _dgrad epilogue on this stream.
    ``side``: an earlier launch's slabs for this launch to sum."""
    dw = dest.view(N, K) if dest is not None else torch.empty((N, K), dtype=torch.float32, device=dy.device)
    ws_n = L.lib().hvit_wgrad_workspace(M, N, K)
    ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=dy.device)
    job = L.SlabSum()

    def launch(sj=side):
        call("hvit_linear_wgrad_defer", dt, dy.data_ptr(), x.data_ptr(), M, N, K, dw.data_ptr(), ws.data_ptr(), ws_n,
             C.byref(sj.job) if sj is not None else None, C.byref(job), stream_ptr())

    with timed(tag, 2.0 * M * N * K):
        launch()
    # (the isolated replay re-runs the GEMM alone: the side job's slabs and destination belong to the step)
    _record(tag, (lambda: launch(None), 2.0 * M * N * K))
    return dw, Deferred(job, ws)


def linear_wgrad(dt, dy, x, M, N, K, bias=False, tag="linear_wgrad", tickets=None, dest=None, out=None):
    """dw [N, K] = dy^T x (f32); with ``bias`` also db [N] = colsum(dy), which
    the bf16 path fuses into the GEMM (db stored right after dw).  ``tickets``
    (a zeroed f32 tensor of at least wgrad_tickets(M, N, K) elements, e.g. a
    slice of the forward's zero pool): the split-K partials are reduced inside
    the GEMM launch (no second launch, no slab re-read pass)."""
    if dest is not None and not bias:  # the parameter's data-parallel bucket slot (grad_dest)
        dw, db = dest.view(N, K), None
    else:
        # (out: a caller's [N*K (+N)] buffer)
        buf = out if out is not None else torch.empty(N * K + (N if bias else 0), dtype=torch.float32,
                                                      device=dy.device)
        dw = buf[:N * K].view(N, K)
        db = buf[N * K:] if bias else None
    ws_n = L.lib().hvit_wgrad_workspace(M, N, K)
    ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=dy.device)

    def launch():
        if tickets is not None:
            call("hvit_linear_wgrad_tk", dt, dy.data_ptr(), x.data_ptr(), M, N, K, dw.data_ptr(), ptr(db),
                 ws.data_ptr(), ws_n, tickets.data_ptr(), tickets.numel(), L.ACC_ZEROED, stream_ptr())
        else:
            call("hvit_linear_wgrad", dt, dy.data_ptr(), x.data_ptr(), M, N, K, dw.data_ptr(), ptr(db),
                 ws.data_ptr(), ws_n, stream_ptr())

    with timed(tag, 2.0 * M * N * K):
        launch()
    _record(tag, (launch, 2.0 * M * N * K))
    return (dw, db) if bias else dw


def linear_wgrad_bias_deferred(dt, dy, x, M, N, K, tag="linear_wgrad", out=None):
    """(dw, db, Deferred or None) of a biased Linear: the tall-skinny kernel's
    [dw | db] slab sum is left to the next linear launch on this stream (pass
    the Deferred as its epilogue side job; dw and db are final once it ran)."""
    if not DEFER:
        dw, db = linear_wgrad(dt, dy, x, M, N, K, bias=True, out=out)
        return dw, db, None
    buf = out if out is not None else torch.empty(N * K + N, dtype=torch.float32, device=dy.device)
    dw, db = buf[:N * K].view(N, K), buf[N * K:]
    ws_n = L.lib().hvit_wgrad_workspace(M, N, K)
    ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=dy.device)
    job = L.SlabSum()

    def launch():
        call("hvit_linear_wgrad_bias_defer", dt, dy.data_ptr(), x.data_ptr(), M, N, K, dw.data_ptr(), db.data_ptr(),
             ws.data_ptr(), ws_n, None, C.byref(job), stream_ptr())

    with timed(tag, 2.0 * M * N * K):
        launch()
    _record(tag, (launch, 2.0 * M * N * K))  # (the isolated replay times the GEMM alone)
    return dw, db, (Deferred(job, ws) if job.n > 0 else None)


def _linear_wgrad_bias_maybe_side(ctx, dt, dy, x, M, N, K):
    """(dw, db, Deferred or None) of a biased Linear (head / skip projections):
    on the side stream when side_ok (complete there), else on the backward's
    stream with the slab sum deferred to the data-gradient launch after it."""
    if not side_ok(ctx.prefs):
        return linear_wgrad_bias_deferred(dt, dy, x, M, N, K)
    buf = torch.empty(N * K + N, dtype=torch.float32, device=dy.device)
    with on_side(dy.device, (dy, x, buf)):
        # the same launches, the slab sum as one of its own (the carried job's order)
        dw, db, j = linear_wgrad_bias_deferred(dt, dy, x, M, N, K, out=buf)
        if j is not None:
            call("hvit_sum_slabs_strided", j.job.src, j.job.splits, j.job.stride, j.job.n, j.job.dst, stream_ptr())
    return dw, db, None


def dropout_scale(g, M, N, drop, rowscale, rps, out, colsum=None):
    """out = rowscale * dropout(g) in out's dtype; colsum (f32 [N], zeroed)
    += column sums of it (per-workgroup partials in a scratch slab)."""
    ws, ws_n = None, 0
    if colsum is not None:
        ws_n = L.lib().hvit_dropout_colsum_ws_elems(N)
        ws = torch.empty(ws_n, dtype=torch.float32, device=g.device)
    with timed("dropout_scale", float(M * N * (g.element_size() + out.element_size()))):  # read g, write out
        call("hvit_dropout_scale", g.data_ptr(), L.dt_of(g), M, N, drop, ptr(rowscale), rps, out.data_ptr(),
             L.dt_of(out), ptr(colsum), ptr(ws), ws_n, stream_ptr())


def linear_wgrad_now(dt, dy, x, M, N, K, tag="vit_linear_wgrad", dest=None, side: Optional["Deferred"] = None):
    """dw [N, K] = dy^T x (f32), complete on the current stream when its
    launches are: the weight gradient with its split-K slab sum (and an incoming
    side job) issued back to back (the side-stream form, where no data-gradient
    launch follows on the same stream to carry the sum)."""
    dw, d = linear_wgrad_deferred(dt, dy, x, M, N, K, tag=tag, dest=dest, side=side)
    if d is not None and d.job.n > 0:
        j = d.job

        def launch():
            call("hvit_sum_slabs_strided", j.src, j.splits, j.stride, j.n, j.dst, stream_ptr())

        with timed(tag, 0.0):
            launch()
        _record(tag, (lambda d=d, dw=dw: launch(), 0.0))  # (d, dw: the slabs and the destination stay alive)
    return dw


# ---------------------------------------------------------------------------
# Weight gradients on a side stream (round 4).  A weight gradient is off the
# critical path of the backward (nothing reads it before the optimizer), so
# the ViT blocks issue theirs on a per-device side stream that forks from the
# backward's stream where its operands are ready; the data-gradient chain
# runs on concurrently.  The side stream is joined back into the stream that
# called backward() by an autograd final callback, before the optimizer, clip
# or the caller can read a gradient; the data-parallel reducer launches its
# bucket all-reduces from the side stream while work is pending there.  A
# weight gradient that a backward ACCUMULATES into an existing .grad stays on
# the backward's stream (autograd reads it right away).  Tensors crossing the
# streams are registered with record_stream, so the caching allocator never
# recycles them under a pending side launch.  Graph capture forks and joins
# the side stream like any other (parallel branches of the captured step).
# Off by default: measured on the MI355X (B=32 graph step, tools/gpu_session.sh
# env:HVIT_SIDE=...), the single-stream step is faster -- 5.62 vs 5.70 ms: the
# data-gradient GEMMs already fill the 256 CUs, so the concurrent weight
# gradients only add their split-K slab sums (a launch each on the side stream,
# where no following launch carries them) and contend for the CUs; fewer
# side-stream splits (HVIT_SIDE_WG 128 / 64) were slower still (5.79 / 6.10).
SIDE = False  # True: weight gradients on the side stream (tests/test_gpu_determinism.py runs both)
# workgroup target of the side stream's linear weight gradients (split-K
# choice; 0 = the library default)
SIDE_WG = 0
_SIDE_STREAMS = {}
_SIDE_OPEN = set()
_SIDE_TASKS = set()  # autograd graph tasks that have the join queued


def _dev_index(dev) -> int:
    return dev.index if dev.index is not None else torch.cuda.current_device()


def side_stream(dev) -> "torch.cuda.Stream":
    i = _dev_index(dev)
    s = _SIDE_STREAMS.get(i)
    if s is None:
        s = _SIDE_STREAMS[i] = torch.cuda.Stream(device=i)
    return s


def side_pending(dev) -> bool:
    """Side-stream work not yet joined back (during a backward)."""
    return _dev_index(dev) in _SIDE_OPEN


def _join_side():
    for i in list(_SIDE_OPEN):
        torch.cuda.current_stream(i).wait_stream(_SIDE_STREAMS[i])
    _SIDE_OPEN.clear()
    _SIDE_TASKS.clear()


class on_side:
    """``with on_side(dev, tensors):`` launches on the device's side stream,
    ordered after everything issued so far on the current stream; ``tensors``
    (produced or consumed across the two streams) are recorded on the side
    stream.  Registers the join for the end of this backward."""

    __slots__ = ("dev", "tensors", "ctx", "wg")

    def __init__(self, dev, tensors=()):
        self.dev, self.tensors = dev, tensors

    def __enter__(self):
        i = _dev_index(self.dev)
        s = side_stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(i))
        _SIDE_OPEN.add(i)
        task = torch._C._current_graph_task_id()
        if task not in _SIDE_TASKS:  # once per backward (also after one that raised before its join)
            _SIDE_TASKS.add(task)
            torch.autograd.Variable._execution_engine.queue_callback(_join_side)
        for t in self.tensors:
            if t is not None:
                t.record_stream(s)
        self.ctx = torch.cuda.stream(s)
        self.ctx.__enter__()
        self.wg = L.lib().hvit_gemm_tune(2, SIDE_WG) if SIDE_WG > 0 else None
        return s

    def __exit__(self, *exc):
        if self.wg is not None:
            L.lib().hvit_gemm_tune(2, self.wg)
        return self.ctx.__exit__(*exc)


def side_ok(prefs) -> bool:
    """The weight gradients of these parameters may go to the side stream: no
    parameter already holds a .grad that this backward would accumulate into."""
    if not SIDE:
        return False
    for r in prefs:
        p = r()
        if p is not None and p.grad is not None:
            return False
    return True


# ---------------------------------------------------------------------------
# Grouped weight gradients (round 6, hvit_linear_wgrad_group).  Each ViT Linear's
# weight gradient is a GEMM with a small output and a long token reduction
# (8,192 tokens at B = 32): alone it fills the chip only by splitting K into
# short slices with f32 partial slabs.  Nothing reads a weight gradient before
# the optimizer, so the ViT blocks' backward queues them instead (the operands
# are kept alive by the queue) and one launch runs the whole queue: every
# 256x256 output tile over the full token range, written once.  The queue is
# flushed (1) by an autograd final callback at the end of the backward, (2) by
# the data-parallel reducer right before it launches a bucket (dp.py), and (3)
# by any caller that needs the gradients earlier (wgrad_flush).  A parameter
# that already holds a .grad (accumulation) is not queued: autograd adds its
# gradient at once.  The tensor handed to autograd is a fresh view of the
# result buffer; the queue holds a different view of the same storage, so
# autograd adopts the handed view as .grad without a copy (a copy made before
# the flush would copy unwritten memory: the flush re-copies such a .grad).
WGRAD_GROUP = True
_WG_QUEUE = {}    # device index -> [(dy, x, dw base, n, k, M, pref, patch, packed)]
_WG_TASKS = set()  # autograd graph tasks that have the flush queued
_WG_TICKETS = {}  # device index -> zeroed uint32 counters (left zeroed by every launch)
WG_FIXUPS = 0  # gradients autograd copied instead of adopting (re-copied by the flush; tests expect none)


def wgrad_group_ok(dt, M, N, K, pref=None) -> bool:
    """The weight gradient dW[N, K] over M tokens may join the group queue."""
    if not WGRAD_GROUP or SIDE or dt != BF16:
        return False
    if pref is not None:
        p = pref()
        if p is not None and p.grad is not None:
            return False
    return bool(L.lib().hvit_linear_wgrad_group_ok(dt, M, N, K))


def wgrad_enqueue(dy, x, M, N, K, dest=None, pref=None, patch=None) -> torch.Tensor:
    """Queue dW[N, K] = dy[M, :N]^T x[M, :K] (bf16 operands, row pitches taken
    from the tensors); returns the f32 gradient tensor, final once the queue
    is flushed.  ``patch`` = (P, weight shape): x is the NHWC feature map of a
    patch embedding (Conv2d k = stride = P) and the result, computed in the
    packed [N][ky][kx][c] order, is unpacked into the torch-layout weight
    gradient by the flush."""
    dev = dy.device
    i = _dev_index(dev)
    # the queue holds the storage's base tensor, autograd gets a view of it: a
    # view keeps its base alive (._base), so holding a view of the RETURNED
    # tensor would count as a second reference to it and make AccumulateGrad
    # copy it (unwritten) instead of adopting it
    base = dest.view(-1) if dest is not None else torch.empty(N * K, dtype=torch.float32, device=dev)
    if patch is not None:
        dw = base.view(patch[1])
        packed = torch.empty(N * K, dtype=torch.float32, device=dev)
    else:
        dw = base.view(N, K)
        packed = None
    q = _WG_QUEUE.setdefault(i, [])
    q.append((dy, x, base, N, K, M, pref, patch, packed))
    task = torch._C._current_graph_task_id()
    if task >= 0 and task not in _WG_TASKS:
        _WG_TASKS.add(task)
        torch.autograd.Variable._execution_engine.queue_callback(_wgrad_flush_all)
    return dw


def _wgrad_flush_all():
    for i in set(_WG_QUEUE) | set(_SIDE_PENDING) | set(_WG_AFTER):
        wgrad_flush(torch.device("cuda", i))
    _WG_TASKS.clear()


# Launches that read queued gradients and were held back until the grouped
# launch (the DP buckets holding ViT weights: dp.GradAllReducer._launch), run
# by the flush right after it, in the order they were deferred.
_WG_AFTER = {}  # device index -> [callable]
WG_LAUNCHES = 0  # grouped launches issued (tests: one per backward)


def wgrad_pending(dev) -> bool:
    """True while weight gradients of ``dev`` wait in the group queue."""
    return bool(_WG_QUEUE.get(_dev_index(dev)))


def wgrad_after_flush(dev, fn) -> None:
    """Run ``fn()`` right after the next flush of ``dev``'s queue."""
    i = _dev_index(dev)
    _WG_AFTER.setdefault(i, []).append(fn)
    task = torch._C._current_graph_task_id()
    if task >= 0 and task not in _WG_TASKS:
        _WG_TASKS.add(task)
        torch.autograd.Variable._execution_engine.queue_callback(_wgrad_flush_all)


# Partial-row sums (Deferred side jobs) whose results were handed to autograd
# before any launch summed them: the next launch that can carry one takes it
# (side_take), the flush points run whatever is left as launches of their own.
_SIDE_PENDING = {}  # device index -> [Deferred]


def side_defer(job, dev):
    i = _dev_index(dev)
    _SIDE_PENDING.setdefault(i, []).append(job)
    task = torch._C._current_graph_task_id()
    if task >= 0 and task not in _WG_TASKS:
        _WG_TASKS.add(task)
        torch.autograd.Variable._execution_engine.queue_callback(_wgrad_flush_all)
    return job


def side_take(job, dev) -> bool:
    """Claim a pending job for a launch about to carry it (False: already run)."""
    q = _SIDE_PENDING.get(_dev_index(dev), [])
    for k, j in enumerate(q):
        if j is job:
            del q[k]
            return True
    return False


def _side_run_pending(i):
    for j in _SIDE_PENDING.pop(i, []):
        call("hvit_sum_slabs_strided", j.job.src, j.job.splits, j.job.stride, j.job.n, j.job.dst, stream_ptr())


def wgrad_flush(dev=None) -> None:
    """Launch every queued weight gradient of ``dev`` (one grouped launch per
    token count) on the current stream."""
    i = _dev_index(dev) if dev is not None else torch.cuda.current_device()
    _side_run_pending(i)
    q = _WG_QUEUE.pop(i, None)
    if q:
        _wgrad_group_launch(i, q)
    for fn in _WG_AFTER.pop(i, []):
        fn()


def _wgrad_group_launch(i, q):
    global WG_LAUNCHES
    d = torch.device("cuda", i)
    tk = _WG_TICKETS.get(i)
    if tk is None:
        tk = _WG_TICKETS[i] = torch.zeros(int(L.lib().hvit_linear_wgrad_group_tickets()), dtype=torch.int32,
                                          device=d)
    ws = torch.empty(int(L.lib().hvit_linear_wgrad_group_ws()), dtype=torch.float32, device=d)
    by_m = {}
    for job in q:
        by_m.setdefault(job[5], []).append(job)
    for M, jobs in by_m.items():
        arr = (L.WgradProb * len(jobs))()
        flops = 0.0
        for j, (dy, x, dw, n, k, _, _, patch, packed) in enumerate(jobs):
            if patch is None:
                arr[j] = L.WgradProb(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), dw.data_ptr(), n, k)
            else:
                _, H, W, C = x.shape
                arr[j] = L.WgradProb(dy.data_ptr(), dy.stride(0), x.data_ptr(), 0, packed.data_ptr(), n, k,
                                     patch[0], H, W, C)
            flops += 2.0 * M * n * k

        def launch(arr=arr, n=len(jobs), M=M, jobs=jobs):
            call("hvit_linear_wgrad_group", BF16, M, arr, n, ws.data_ptr(), ws.numel(), tk.data_ptr(), tk.numel(),
                 stream_ptr())

        with timed("vit_linear_wgrad", flops):
            launch()
        WG_LAUNCHES += 1
        _record("vit_linear_wgrad", (lambda launch=launch, ws=ws: launch(), flops))
    for dy, x, dw, n, k, _, pref, patch, packed in q:
        if patch is not None:  # [co][ky][kx][c] -> torch's [co][c][ky][kx]
            co, ci, ks, _ = patch[1]
            call("hvit_conv_weight_unpack", packed.data_ptr(), co, ci, ks, dw.data_ptr(), stream_ptr())
        p = pref() if pref is not None else None
        if p is not None and p.grad is not None and p.grad.data_ptr() != dw.data_ptr():
            # autograd copied the handed tensor before it was written
            global WG_FIXUPS
            WG_FIXUPS += 1
            p.grad.copy_(dw.view(p.grad.shape))


class Deferred:
    """A weight gradient whose split-K slab sum is handed to the next linear
    launch on the stream (hvit_linear_wgrad_defer): ``job`` goes into that
    launch's epilogue ``side``; ``ws`` (the slabs) is held until it is enqueued."""

    __slots__ = ("job", "ws")

    def __init__(self, job, ws):
        self.job, self.ws = job, ws


def epilogue(act=L.ACT_NONE, out2=None, aux=None, drop=None, resid=None, rowscale=None, rps=1, rowadd=None,
             rowadd_rows=1, colsum=None, side: Optional[Deferred] = None):
    e = L.Epilogue()
    if side is not None:
        e.side = side.job
    e.act = act
    e.out2 = ptr(out2)
    e.out2_dt = L.dt_of(out2) if out2 is not None else 0
    e.aux = ptr(aux)
    e.aux_dt = L.dt_of(aux) if aux is not None else 0
    e.dropout = drop if drop is not None else L.dropout()
    e.resid = ptr(resid)
    e.rowscale = ptr(rowscale)
    e.rows_per_sample = rps
    e.rowadd = ptr(rowadd)
    e.rowadd_rows = rowadd_rows
    e.colsum = ptr(colsum)
    return e


def geom(src1, C1, src2, C2, N, Hs, Ws, U, KS, stride, pad, Cout) -> L.ConvGeom:
    return L.ConvGeom(ptr(src1), C1, ptr(src2), C2, N, Hs, Ws, U, KS, stride, pad, Cout)


def conv_wgrad(dt, g: L.ConvGeom, dz, wshape, dest=None) -> torch.Tensor:
    """Conv weight gradient in the Parameter's layout [Cout][Cin][KS][KS]: the
    split-K slab sum writes that order directly (hvit_conv_wgrad_torch)."""
    co, ci, ks, _ = wshape
    dw = dest if dest is not None else torch.empty(wshape, dtype=torch.float32, device=dz.device)
    dwp = torch.empty(co * ci * ks * ks, dtype=torch.float32, device=dz.device)
    ws_n = L.lib().hvit_conv_wgrad_workspace(g)
    ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=dz.device)
    P = dz.numel() // co  # output pixels

    def launch():
        call("hvit_conv_wgrad_torch", dt, g, dz.data_ptr(), dw.data_ptr(), dwp.data_ptr(), ws.data_ptr(), ws_n,
             stream_ptr())

    with timed("conv_wgrad", 2.0 * P * co * ci * ks * ks):
        launch()
    _record("conv_wgrad", (launch, 2.0 * P * co * ci * ks * ks))
    return dw.view(wshape)


def _conv_wgrad_maybe_side(ctx, dt, g, dz, w, srcs):
    """A conv weight gradient on the side stream when side_ok (its operands:
    dz and the conv input tensors behind the geometry's raw pointers), else on
    the backward's stream; into the parameter's data-parallel slot when one is
    published."""
    dest = grad_dest(*ctx.wid)
    if not side_ok(ctx.prefs):
        return conv_wgrad(dt, g, dz, w.shape, dest)
    if dest is None:
        dest = torch.empty(w.shape, dtype=torch.float32, device=dz.device)
    with on_side(dz.device, (dz, dest) + tuple(srcs)):
        conv_wgrad(dt, g, dz, w.shape, dest)
    return dest.view(w.shape)


@dataclass
class Drop:
    """A dropout site: probability, seed and site id.  ``seed_t`` (optional): the
    forward's device seed word (HybridViT._forward_seed); the kernels then use
    ``seed ^ seed_t[0]``, read on the device, so a captured train step draws new
    masks on every replay."""
    p: float = 0.0
    seed: int = 0
    site: int = 0
    seed_t: Optional[torch.Tensor] = None
    # DropPath sites only: this block's [2B] multipliers, already drawn by the
    # forward's one droppath_scales_all launch (used instead of a launch of its own)
    pre: Optional[torch.Tensor] = field(default=None, compare=False, repr=False)

    def c(self):
        return L.dropout(self.p, self.seed, self.site, self.seed_t)


# ----------------------------------------------------------------------------
class CastFn(torch.autograd.Function):
    """Input cast to the compute dtype (gradient cast back)."""

    @staticmethod
    def forward(ctx, x, dt):
        ctx.src_dt = L.dt_of(x)
        return cast(x, dt)

    @staticmethod
    def backward(ctx, g):
        return cast(g, ctx.src_dt), None


SKIPGRAD = True  # False: autograd adds the skip gradients
# the gradient at a LayerNorm output (a linear's data gradient) in the compute
# dtype; False: f32 (the round-5 form)
LN_DY_LOW = True


class SkipGrad:
    """The skip gradient of one encoder output, handed from its SkipFn to its
    other consumer (the next encoder block or the patch embedding) instead of
    being summed by autograd (hybrid_vit.py:303-305, 376-389: an encoder output
    feeds both).  SkipFn's backward offers its gradient at decoder resolution,
    before the bilinear backward; the other consumer's backward then runs that
    bilinear backward in accumulate mode straight into its own input gradient,
    so no separate add of two full-resolution tensors is launched.  Backward
    order makes the offer come first (the decoder's backward completes before
    the ViT's, which precedes the encoder's); if the consumer drained first,
    SkipFn returns its gradient to autograd as usual."""

    __slots__ = ("dr", "meta", "closed")

    def __init__(self):
        self.dr, self.meta, self.closed = None, None, False

    def offer(self, dr, meta) -> bool:
        if self.closed:
            return False
        self.dr, self.meta = dr, meta
        return True

    def drain(self, de):
        """Add the offered gradient into ``de`` (the consumer's NHWC input gradient)."""
        self.closed = True
        if self.dr is None:
            return
        N, Ho, Wo, Ce, He, We, dt = self.meta
        assert tuple(de.shape) == (N, He, We, Ce) and de.is_contiguous(), (de.shape, self.meta)
        call("hvit_bilinear_bwd", self.dr.data_ptr(), dt, N, Ho, Wo, Ce, He, We, de.data_ptr(), L.dt_of(de), 1,
             stream_ptr())
        self.dr = None


class ConvBNActFn(torch.autograd.Function):
    """[nearest up U] -> Conv KSxKS (no bias) over concat(x1, x2) -> BatchNorm2d
    -> ReLU -> Dropout2d -> [MaxPool 2]  (ConvBlock components.py:15-99,
    TransposeConvBlock components.py:102-192 with the decoder concat of
    hybrid_vit.py:389).  NHWC in / out."""

    @staticmethod
    def forward(ctx, x1, x2, w, gamma, beta, rmean, rvar, nbt, U, pool, training, drop: Drop, momentum, eps, dt,
                sg: Optional[SkipGrad] = None, nograd: bool = False):
        N, Hs, Ws, C1 = x1.shape
        C2 = x2.shape[3] if x2 is not None else 0
        Cout, Cin, KS, _ = w.shape
        assert Cin == C1 + C2, (Cin, C1, C2)
        H, W = Hs * U, Ws * U
        dev = x1.device
        s = stream_ptr()
        g = geom(x1, C1, x2, C2, N, Hs, Ws, U, KS, 1, KS // 2, Cout)
        mean = torch.empty(Cout, dtype=torch.float32, device=dev)
        invstd = torch.empty_like(mean)
        P = N * H * W
        es = 4 if dt == F32 else 2
        cflops = 2.0 * P * Cout * Cin * KS * KS
        pooled = (pool == 2 and dt == BF16 and C1 % 64 == 0 and C2 % 64 == 0 and H % 2 == 0 and W % 2 == 0
                  and Cout % 4 == 0)
        if nograd and not training and (pool == 1 or pooled) and EVALFOLD:
            # eval, no backward (the caller ran outside grad mode): BatchNorm folded into the conv weights and bias, ReLU
            # in the conv epilogue (Dropout2d is the identity): z is never stored.  A pooling block (enc1) walks
            # its output pixels window by window and keeps each 2x2 window's maximum in the epilogue.
            folded = _prep_get(w, 3, dt)  # (the module forward's weight_prep launch folded it)
            if folded is not None:
                wf, bias = folded
            else:
                call("hvit_bn_eval_prep", rmean.data_ptr(), rvar.data_ptr(), Cout, eps, mean.data_ptr(),
                     invstd.data_ptr(), s)
                wf = _empty((w.numel(),), dt, dev)
                bias = torch.empty(Cout, dtype=torch.float32, device=dev)
                call("hvit_bn_fold", w.detach().contiguous().data_ptr(), Cout, Cin, KS, mean.data_ptr(),
                     invstd.data_ptr(), gamma.detach().contiguous().data_ptr(),
                     beta.detach().contiguous().data_ptr(), wf.data_ptr(), dt, bias.data_ptr(), s)
            y = _empty((N, H // pool, W // pool, Cout), dt, dev)
            with timed("conv_fwd", cflops):
                call("hvit_conv_fwd", dt, g, wf.data_ptr(), bias.data_ptr(), y.data_ptr(), dt, None,
                     epilogue(act=L.ACT_RELU_POOL2 if pool == 2 else L.ACT_RELU), s)
            return y
        wp = pack_conv(w, 0, dt)
        z = _empty((N, H, W, Cout), dt, dev)
        if training:
            tr = L.lib().hvit_conv_bn_tile_rows(C.byref(g))  # rows per BN partial tile
            nt = (P + tr - 1) // tr
            part = torch.empty((nt, Cout, 2), dtype=torch.float32, device=dev)
            with timed("conv_fwd", cflops):
                call("hvit_conv_fwd", dt, g, wp.data_ptr(), None, z.data_ptr(), dt, part.data_ptr(), None, s)
            call("hvit_bn_finalize", part.data_ptr(), nt, tr, P, Cout, mean.data_ptr(), invstd.data_ptr(),
                 ptr(rmean), ptr(rvar), ptr(nbt), momentum, eps, s)
        else:
            with timed("conv_fwd", cflops):
                call("hvit_conv_fwd", dt, g, wp.data_ptr(), None, z.data_ptr(), dt, None, None, s)
            call("hvit_bn_eval_prep", rmean.data_ptr(), rvar.data_ptr(), Cout, eps, mean.data_ptr(),
                 invstd.data_ptr(), s)
        y = _empty((N, H // pool, W // pool, Cout), dt, dev)
        dr = drop.c() if training else L.dropout()
        with timed("bn_act_fwd", float(P * Cout * es * (1 + 1.0 / (pool * pool)))):  # read z, write y
            call("hvit_bn_act_fwd", dt, z.data_ptr(), N, H, W, Cout, mean.data_ptr(), invstd.data_ptr(),
                 gamma.data_ptr(), beta.data_ptr(), dr, pool, y.data_ptr(), dt, s)
        ctx.save_for_backward(x1, x2, w, gamma, beta)
        ctx.wid = (id(w), tuple(w.shape))
        ctx.prefs = (weakref.ref(w),)
        ctx.z, ctx.mean, ctx.invstd = z, mean, invstd
        ctx.meta = (U, pool, training, dr, dt)
        ctx.sg = sg
        return y

    @staticmethod
    def backward(ctx, dy):
        x1, x2, w, gamma, beta = ctx.saved_tensors
        U, pool, training, dr, dt = ctx.meta
        z = ctx.z
        N, H, W, Cout = z.shape
        Hs, Ws, C1 = x1.shape[1], x1.shape[2], x1.shape[3]
        C2 = x2.shape[3] if x2 is not None else 0
        KS = w.shape[2]
        dev = z.device
        s = stream_ptr()
        dy = dy.contiguous()
        dz = _empty(z.shape, dt, dev)
        # [dbeta | dgamma] followed by per-workgroup partial rows (plain stores: no zeroing)
        sums = torch.empty(L.lib().hvit_bn_act_bwd_sums_elems(Cout), dtype=torch.float32, device=dev)
        with timed("bn_act_bwd", float(2 * z.numel() * z.element_size() + dy.numel() * dy.element_size())):
            call("hvit_bn_act_bwd", dt, z.data_ptr(), N, H, W, Cout, ctx.mean.data_ptr(), ctx.invstd.data_ptr(),
                 gamma.data_ptr(), beta.data_ptr(), dr, pool, dy.data_ptr(), L.dt_of(dy), int(training),
                 dz.data_ptr(), dt, sums.data_ptr(), L.ACC_ZEROED, s)
        dbeta, dgamma = sums[:Cout], sums[Cout:2 * Cout]
        g = geom(x1, C1, x2, C2, N, Hs, Ws, U, KS, 1, KS // 2, Cout)
        dw = _conv_wgrad_maybe_side(ctx, dt, g, dz, w, (x1, x2))
        dx1 = dx2 = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            wd = pack_conv(w, 1, dt)
            du = _empty((N, H, W, C1 + C2), dt, dev)
            with timed("conv_dgrad", 2.0 * N * H * W * Cout * (C1 + C2) * KS * KS):
                call("hvit_conv_dgrad", dt, g, dz.data_ptr(), wd.data_ptr(), du.data_ptr(), dt, s)
            if U == 1 and C2 == 0:
                dx1 = du
                if ctx.sg is not None:
                    ctx.sg.drain(dx1)
            else:
                dx1 = _empty((N, Hs, Ws, C1), dt, dev)
                dx2 = _empty((N, Hs, Ws, C2), dt, dev) if C2 else None
                call("hvit_upsample_split_bwd", du.data_ptr(), dt, N, Hs, Ws, U, C1, C2, dx1.data_ptr(), dt,
                     ptr(dx2), dt, s)
        return (dx1, dx2, dw, dgamma, dbeta) + (None,) * 12


# Path switches (module attributes; the tests flip some of them to compare the
# fused form with the separate one).  Round 6 retired their environment reads:
# every A/B they served is concluded.
C1BLOCK = True  # False: the unfused conv + bn_act path
EVALFOLD = True  # False: eval convs keep z + bn_act
KEEPBITS = True  # False: the attention backward re-hashes dropout
LNDROP = True  # False: separate LayerNorm backward and dropout pass
# False: ViT weight gradients reduce their split-K slabs in a launch of their
# own and the qkv bias gradient is a column reduction of dqkv
DEFER = True
# False: the qkv bias gradient by a column reduction of dqkv after the attention
# backward (instead of the backward's partial rows)
ATTN_DB = True
# the fc1 forward folds its dropout multiplier into the stored gelu'(h)
# (GELU_DUAL_DK: dh = dA * [keep * scale * gelu'(h)]), so the fc2 data-gradient
# epilogue multiplies without re-hashing the mask.  False: the round-5 form
# (gelu'(h) stored, the mask re-hashed in the backward)
FC1_FOLD = True


def c1block_ok(x1, x2, w, U, pool) -> bool:
    """The fused first block (hvit_c1block_*) applies: a single-channel input that
    needs no gradient, 3x3 same conv, power-of-two Cout <= 256, rows that fit
    the kernel's LDS staging."""
    if not C1BLOCK or x2 is not None or U != 1 or pool not in (1, 2) or x1.requires_grad:
        return False
    co, ci, ks, _ = w.shape
    return ci == 1 and ks == 3 and 8 <= co <= 256 and co & (co - 1) == 0 and x1.shape[2] + 2 <= 8192 // (pool + 2)


class C1BlockFn(torch.autograd.Function):
    """The first encoder ConvBlock (hybrid_vit.py:196-208 -> components.py:55-85,
    Cin = 1) fused so that the conv output z never reaches HBM: BatchNorm
    statistics, the BN/ReLU/Dropout2d/MaxPool apply, and the backward
    (BN backward + conv weight gradient, dz kept in registers) each recompute
    z from the single-channel input (csrc/c1block.hip).  Same arguments and
    result as ConvBNActFn for that block; the input gets no gradient."""

    @staticmethod
    def forward(ctx, x1, w, gamma, beta, rmean, rvar, nbt, pool, training, drop: Drop, momentum, eps, dt):
        N, H, W, _ = x1.shape
        Cout = w.shape[0]
        dev = x1.device
        s = stream_ptr()
        wp = pack_conv(w, 0, dt)
        g = geom(x1, 1, None, 0, N, H, W, 1, 3, 1, 1, Cout)
        mean = torch.empty(Cout, dtype=torch.float32, device=dev)
        invstd = torch.empty_like(mean)
        P = N * H * W
        es = 4 if dt == F32 else 2
        if training:
            tr = L.lib().hvit_conv_bn_tile_rows(C.byref(g))
            nt = (P + tr - 1) // tr
            part = torch.empty((nt, Cout, 2), dtype=torch.float32, device=dev)
            with timed("c1block_stats", float(P * x1.element_size())):  # reads x
                call("hvit_c1block_stats", dt, g, wp.data_ptr(), part.data_ptr(), s)
            call("hvit_bn_finalize", part.data_ptr(), nt, tr, P, Cout, mean.data_ptr(), invstd.data_ptr(),
                 ptr(rmean), ptr(rvar), ptr(nbt), momentum, eps, s)
        else:
            call("hvit_bn_eval_prep", rmean.data_ptr(), rvar.data_ptr(), Cout, eps, mean.data_ptr(),
                 invstd.data_ptr(), s)
        y = _empty((N, H // pool, W // pool, Cout), dt, dev)
        dr = drop.c() if training else L.dropout()
        with timed("c1block_fwd", float(P * x1.element_size() + y.numel() * es)):  # read x, write y
            call("hvit_c1block_fwd", dt, g, wp.data_ptr(), mean.data_ptr(), invstd.data_ptr(), gamma.data_ptr(),
                 beta.data_ptr(), dr, pool, y.data_ptr(), dt, s)
        ctx.save_for_backward(x1, w, gamma, beta)
        ctx.mean, ctx.invstd = mean, invstd
        ctx.meta = (pool, training, dr, dt)
        return y

    @staticmethod
    def backward(ctx, dy):
        x1, w, gamma, beta = ctx.saved_tensors
        pool, training, dr, dt = ctx.meta
        N, H, W, _ = x1.shape
        Cout = w.shape[0]
        dev = x1.device
        s = stream_ptr()
        dy = dy.contiguous()
        g = geom(x1, 1, None, 0, N, H, W, 1, 3, 1, 1, Cout)
        wp = pack_conv(w, 0, dt)
        sums = torch.empty(2 * Cout, dtype=torch.float32, device=dev)  # [dbeta | dgamma]
        dwp = torch.empty(w.numel(), dtype=torch.float32, device=dev)
        ws_n = L.lib().hvit_c1block_bwd_ws(C.byref(g), pool)
        ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=dev)
        passes = 2

        def launch():
            call("hvit_c1block_bwd", dt, g, wp.data_ptr(), ctx.mean.data_ptr(), ctx.invstd.data_ptr(),
                 gamma.data_ptr(), beta.data_ptr(), dr, pool, dy.data_ptr(), L.dt_of(dy), int(training),
                 sums.data_ptr(), L.ACC_ZEROED, dwp.data_ptr(), ws.data_ptr(), ws_n, s)

        with timed("c1block_bwd", float(passes * (dy.numel() * dy.element_size() + x1.numel() * x1.element_size()))):
            launch()
        dbeta, dgamma = sums[:Cout], sums[Cout:2 * Cout]
        # mode-0 packing of a Cin = 1 weight is the torch layout [Cout][1][3][3]
        return (None, dwp.view(w.shape), dgamma, dbeta) + (None,) * 9


class PatchEmbedFn(torch.autograd.Function):
    """PatchEmbedding conv k=s=P + flatten/transpose (components.py:282-307),
    + pos_embed[:, :N] and dropout (PositionalEncoding components.py:371-386).
    NHWC feature map -> f32 tokens [B, N, D]."""

    @staticmethod
    def forward(ctx, feat, w, b, pos, Pp, drop: Drop, training, dt, sg: Optional[SkipGrad] = None):
        N, H, W, C = feat.shape
        D = w.shape[0]
        Hp, Wp = H // Pp, W // Pp
        Nt = Hp * Wp
        if pos is not None and Nt > pos.shape[1]:
            raise ValueError(f"hvit: {Nt} patches exceed the positional table ({pos.shape[1]})")
        dev = feat.device
        s = stream_ptr()
        wp = pack_conv(w, 0, dt)
        x0 = torch.empty((N, Nt, D), dtype=torch.float32, device=dev)
        g = geom(feat, C, None, 0, N, H, W, 1, Pp, Pp, 0, D)
        dr = drop.c() if training else L.dropout()
        e = epilogue(drop=dr, rowadd=pos, rowadd_rows=Nt)
        call("hvit_conv_fwd", dt, g, wp.data_ptr(), b.data_ptr(), x0.data_ptr(), F32, None, e, s)
        ctx.save_for_backward(feat, w)
        ctx.wid = (id(w), tuple(w.shape))
        ctx.prefs = (weakref.ref(w),)
        ctx.wp = wp
        ctx.meta = (Pp, dr, dt, Nt, None if pos is None else pos.shape)
        ctx.sg = sg
        ctx.zs = _zs(ctx, D)
        return x0

    @staticmethod
    def backward(ctx, dx0):
        feat, w = ctx.saved_tensors
        Pp, dr, dt, Nt, pshape = ctx.meta
        N, H, W, C = feat.shape
        D = w.shape[0]
        dev = feat.device
        s = stream_ptr()
        dx0 = dx0.contiguous()
        M = N * Nt
        gd = _empty((M, D), dt, dev)
        db = ctx.zs.take(dev)  # patch-embed bias grad: column sums fused into the dropout pass
        dropout_scale(dx0, M, D, dr, None, 1, gd, db)
        dpos = None
        if pshape is not None:
            dpos = torch.zeros(pshape, dtype=torch.float32, device=dev)
            call("hvit_reduce_rows", gd.data_ptr(), dt, N, Nt * D, Nt * D, 1, dpos.data_ptr(), s)
        g = geom(feat, C, None, 0, N, H, W, 1, Pp, Pp, 0, D)
        if (not SIDE and dt == BF16 and wgrad_group_ok(dt, M, D, Pp * Pp * C, ctx.prefs[0])
                and L.lib().hvit_linear_wgrad_group_patch_ok(dt, M, D, Pp, H, W, C)):
            # queued with the ViT blocks' weight gradients (one grouped launch)
            dw = wgrad_enqueue(gd, feat, M, D, Pp * Pp * C, grad_dest(*ctx.wid), ctx.prefs[0],
                               patch=(Pp, tuple(w.shape)))
        else:
            dw = _conv_wgrad_maybe_side(ctx, dt, g, gd, w, (feat,))
        dfeat = None
        if ctx.needs_input_grad[0]:
            dfeat = _empty(feat.shape, dt, dev)
            call("hvit_conv_dgrad", dt, g, gd.data_ptr(), ctx.wp.data_ptr(), dfeat.data_ptr(), dt, s)
            if ctx.sg is not None:
                ctx.sg.drain(dfeat)
        # the ViT blocks' backward is done: their grouped weight gradients go now rather than at the end of
        # backward, so the DP buckets holding them (deferred until the flush) reduce under the encoder backward
        wgrad_flush(dev)
        return dfeat, dw, db, dpos, None, None, None, None, None


class PosDropFn(torch.autograd.Function):
    """tokens + pos_embed[:, :N] and dropout (PositionalEncoding components.py:371-386)
    on tokens handed in from outside the fused patch-embed GEMM: forward_transformer's
    entry (hybrid_vit.py:309-333) and the CLS-token layout.  Same counter-hash mask
    (site 200, element index over [B*N, D]) as PatchEmbedFn's epilogue.  f32 [B, N, D]."""

    @staticmethod
    def forward(ctx, x, pos, drop: Drop, training):
        B, N, D = x.shape
        if N > pos.shape[1]:
            raise ValueError(f"hvit: {N} tokens exceed the positional table ({pos.shape[1]})")
        t = x.float() + pos[:, :N]
        dr = drop.c() if training else L.dropout()
        out = torch.empty_like(t)
        dropout_scale(t, B * N, D, dr, None, 1, out)
        ctx.meta = (dr, pos.shape, N, x.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        dr, pshape, N, xdt = ctx.meta
        B, _, D = g.shape
        gd = torch.empty((B, N, D), dtype=torch.float32, device=g.device)
        dropout_scale(g.contiguous(), B * N, D, dr, None, 1, gd)
        dpos = torch.zeros(pshape, dtype=torch.float32, device=g.device)
        call("hvit_reduce_rows", gd.data_ptr(), F32, B, N * D, N * D, 1, dpos.data_ptr(), stream_ptr())
        return gd.to(xdt), dpos, None, None


def _ln(x2d, gw, gb, dt):
    M, D = x2d.shape
    y = _empty((M, D), dt, x2d.device)
    mean = torch.empty(M, dtype=torch.float32, device=x2d.device)
    rstd = torch.empty_like(mean)
    with timed("layernorm_fwd", float(M * D * (4 + y.element_size()) + 8 * M)):  # read x f32, write y, stats
        call("hvit_layernorm_fwd", x2d.data_ptr(), gw.data_ptr(), gb.data_ptr(), M, D, 1e-5, y.data_ptr(), dt,
             mean.data_ptr(), rstd.data_ptr(), stream_ptr())
    return y, mean, rstd


_LN_SLAB = True


def _ln_bwd(dy, x, mean, rstd, gw, resid, zs: ZSlot):
    """zs: a zslot(2 * D) registered in the forward (dgamma | dbeta)."""
    M, D = x.shape
    dx = torch.empty((M, D), dtype=torch.float32, device=x.device)
    acc = zs.take(x.device)
    dgw, dgb = acc[:D], acc[D:2 * D]
    ws, ws_n = None, 0
    if _LN_SLAB:  # per-workgroup dgamma/dbeta slab + one column reduction (no same-address atomics)
        ws_n = L.lib().hvit_layernorm_bwd_ws_elems(M, D)
        ws = torch.empty(ws_n, dtype=torch.float32, device=x.device)
    # read dy, x f32 (+ resid f32), write dx f32
    with timed("layernorm_bwd", float(M * D * (dy.element_size() + 8 + (4 if resid is not None else 0)))):
        call("hvit_layernorm_bwd", dy.data_ptr(), L.dt_of(dy), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
             gw.data_ptr(), M, D, ptr(resid), dx.data_ptr(), dgw.data_ptr(), dgb.data_ptr(), ptr(ws), ws_n,
             L.ACC_ZEROED, stream_ptr())
    return dx, dgw, dgb


def _ln_bwd_drop(dy, x, mean, rstd, gw, resid, zs: ZSlot, drop, rowscale, rps, g_dt, defer=False):
    """_ln_bwd fused with dropout_scale of its output: returns dx (f32), dgamma,
    dbeta, g = rowscale * dropout(dx) in g_dt and colsum(g).  zs: a zslot(3 * D)
    (dgamma | dbeta | colsum).  ``defer``: the [dgamma | dbeta | colsum] row sum
    is left to a later launch -- a sixth value, the Deferred job to pass as its
    side job (the three results are final once that launch is)."""
    M, D = x.shape
    dx = torch.empty((M, D), dtype=torch.float32, device=x.device)
    g = _empty((M, D), g_dt, x.device)
    acc = zs.take(x.device) if not defer else torch.empty(3 * D, dtype=torch.float32, device=x.device)
    ws_n = L.lib().hvit_layernorm_bwd_drop_ws_elems(M, D)
    ws = torch.empty(ws_n, dtype=torch.float32, device=x.device)
    es = g.element_size()
    with timed("layernorm_bwd", float(M * D * (dy.element_size() + 8 + (4 if resid is not None else 0) + es))):
        call("hvit_layernorm_bwd_drop", dy.data_ptr(), L.dt_of(dy), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
             gw.data_ptr(), M, D, ptr(resid), dx.data_ptr(), acc.data_ptr(), drop, ptr(rowscale), rps, g.data_ptr(),
             g_dt, ws.data_ptr(), ws_n, L.ACC_DEFER if defer else L.ACC_ZEROED, stream_ptr())
    out = (dx, acc[:D], acc[D:2 * D], g, acc[2 * D:3 * D])
    if defer:
        rows = ws_n // (3 * D)
        out += (Deferred(L.SlabSum(ws.data_ptr(), acc.data_ptr(), 3 * D, 3 * D, rows), (ws, acc)),)
    return out


class GradHandoff:
    """Block l's MLP-branch dropout (its fc2 input gradient g2 = DropPath *
    Dropout of the incoming gradient, attention.py:210-211) computed by the
    NEXT consumer of block l's output -- block l+1's LN1 backward or the head's
    final-LN backward -- while that gradient is in its registers
    (_ln_bwd_drop).  Block l's forward fills the dropout config; the consumer's
    backward fills g and colsum; block l's backward (which runs after it) uses
    them instead of a dropout_scale pass.  Unfilled: block l falls back."""

    __slots__ = ("drop", "rowscale", "rps", "dt", "g", "colsum", "job")

    def __init__(self):
        self.drop = self.rowscale = self.rps = self.dt = self.g = self.colsum = self.job = None

    def fuse(self, dy, x, mean, rstd, gw, resid, zs, lnrefs=()):
        """The consumer's LN backward with this handoff's dropout fused; returns
        (dx, dgamma, dbeta) like _ln_bwd.  Under the grouped weight gradients its
        [dgamma | dbeta | colsum] partial-row sum is deferred (``job``) to block
        l's first data-gradient launch, which carries it as a side job (a pending
        side job: every flush point runs it if no launch has).  ``lnrefs``: the
        LayerNorm's parameters -- not deferred when one of them already holds a
        .grad (autograd would add the unwritten sums at once)."""
        if WGRAD_GROUP and not SIDE and dy.is_cuda and lnrefs and all(
                (r() is None or r().grad is None) for r in lnrefs):
            dx, dgw, dgb, g, cs, job = _ln_bwd_drop(dy, x, mean, rstd, gw, resid, zs, self.drop, self.rowscale,
                                                    self.rps, self.dt, defer=True)
            self.job = side_defer(job, dy.device)
        else:
            dx, dgw, dgb, g, cs = _ln_bwd_drop(dy, x, mean, rstd, gw, resid, zs, self.drop, self.rowscale, self.rps,
                                               self.dt)
        self.g, self.colsum = g, cs
        return dx, dgw, dgb


def droppath_scales(B, p, seed, dev):
    """DropPath (components.py:407-427) multipliers of a block's two residual
    branches from one launch: keep(seed, site 1, b) for the attention branch,
    keep(seed, site 1, B + b) for the MLP branch.  ``seed``: an int, or a Drop
    whose (seed, seed_t) are used (site 1, its p ignored)."""
    if p <= 0:
        return None, None
    if isinstance(seed, Drop) and seed.pre is not None and seed.pre.numel() == 2 * B:
        return seed.pre[:B], seed.pre[B:]
    out = torch.empty(2 * B, dtype=torch.float32, device=dev)
    d = L.dropout(p, seed.seed, 1, seed.seed_t) if isinstance(seed, Drop) else L.dropout(p, seed, 1)
    call("hvit_droppath_scale", 2 * B, d, out.data_ptr(), stream_ptr())
    return out[:B], out[B:]


def droppath_scales_all(B, sites, dev):
    """droppath_scales for several blocks from ONE launch: ``sites`` are the
    blocks' (p, Drop) pairs (p > 0); each Drop's ``pre`` is set to its [2B]
    multipliers (the same values droppath_scales(B, p, drop) draws)."""
    sites = [(p, d) for p, d in sites if p > 0]
    if not sites:
        return
    out = torch.empty((len(sites), 2 * B), dtype=torch.float32, device=dev)
    for k in range(0, len(sites), 32):
        part = sites[k:k + 32]
        arr = (L.Dropout * len(part))()
        keep = []
        for i, (p, d) in enumerate(part):
            arr[i] = L.dropout(p, d.seed, 1, d.seed_t)
            keep.append(arr[i])
        call("hvit_droppath_scales", 2 * B, len(part), arr, out[k].data_ptr(), stream_ptr())
    for i, (_, d) in enumerate(sites):
        d.pre = out[i]


class ViTBlockFn(torch.autograd.Function):
    """Pre-norm TransformerEncoderBlock (attention.py:176-213):
    x1 = x + DropPath(Dropout(proj(MHSA(LN1 x))));  x2 = x1 + DropPath(FFN(LN2 x1))
    with MHSA attention.py:65-115 and FeedForward components.py:223-241.
    f32 residual stream [B, N, D] in and out."""

    @staticmethod
    def forward(ctx, x, n1w, n1b, qkvw, qkvb, pw, pb, n2w, n2b, f1w, f1b, f2w, f2b, H, drops, dpr, training,
                dt, want_probs, attn_fp8=False, ho_in: Optional[GradHandoff] = None,
                ho_out: Optional[GradHandoff] = None, nograd: bool = False):
        B, Nt, D = x.shape
        M = B * Nt
        hd = D // H
        hid = f1w.shape[0]
        dev = x.device
        s = stream_ptr()
        scale = hd ** -0.5
        x2d = x.contiguous().view(M, D)
        d_attn, d_proj, d_fc1, d_fc2, dp_seed = drops if training else (Drop(),) * 4 + (0,)
        rs1, rs2 = droppath_scales(B, dpr if training else 0.0, dp_seed, dev)
        xn1, m1, r1 = _ln(x2d, n1w, n1b, dt)
        Wqkv = cast(qkvw, dt)
        qkv = _empty((M, 3 * D), dt, dev)
        _launch("vit_linear_fwd", 2.0 * M * 3 * D * D,
                lambda e, st=s: call("hvit_linear_fwd", dt, xn1.data_ptr(), Wqkv.data_ptr(), qkvb.data_ptr(), M, 3 * D, D,
                               qkv.data_ptr(), dt, e, st))
        o = _empty((M, D), dt, dev)
        lse = torch.empty((B, H, Nt), dtype=torch.float32, device=dev)
        kbits = None
        probs = torch.empty((B, H, Nt, Nt), dtype=torch.float32, device=dev) if want_probs else None
        if attn_fp8 and not want_probs:
            # fp8 (e4m3) QK^T / PV forward (BASELINE config 5); the backward
            # below is the bf16 kernel, recomputing P from this lse and reading
            # the dropout decisions the fp8 forward kept (same keep-bit layout)
            if dt != BF16:
                raise ValueError("hvit: the fp8 attention path runs inside the bf16 model (precision='bf16')")
            if d_attn.p > 0 and KEEPBITS and L.lib().hvit_mhsa_keep_bits_used(dt, Nt, hd):
                kbits = torch.empty(L.lib().hvit_mhsa_keep_bits_elems(B, Nt, H), dtype=torch.int32, device=dev)
            with timed("attn_fwd", 4.0 * B * H * Nt * Nt * hd):
                call("hvit_mhsa_fwd_fp8_kb", qkv.data_ptr(), B, Nt, H, hd, scale, d_attn.c(), o.data_ptr(),
                     lse.data_ptr(), ptr(kbits), s)
        elif probs is None and d_attn.p > 0 and KEEPBITS and L.lib().hvit_mhsa_keep_bits_used(dt, Nt, hd):
            # the dropout decisions are kept (1 bit per score) so the backward does not re-hash them
            # (only for the shapes whose kernels use them: the buffer grows as N^2)
            kbits = torch.empty(L.lib().hvit_mhsa_keep_bits_elems(B, Nt, H), dtype=torch.int32, device=dev)
            with timed("attn_fwd", 4.0 * B * H * Nt * Nt * hd):
                call("hvit_mhsa_fwd_kb", dt, qkv.data_ptr(), B, Nt, H, hd, scale, d_attn.c(), o.data_ptr(),
                     lse.data_ptr(), kbits.data_ptr(), s)
        else:
            with timed("attn_fwd", 4.0 * B * H * Nt * Nt * hd):
                call("hvit_mhsa_fwd", dt, qkv.data_ptr(), B, Nt, H, hd, scale, d_attn.c(), o.data_ptr(),
                     lse.data_ptr(), ptr(probs), s)
        Wp = cast(pw, dt)
        x1 = torch.empty((M, D), dtype=torch.float32, device=dev)
        _launch("vit_linear_fwd", 2.0 * M * D * D,
                lambda e, st=s: call("hvit_linear_fwd", dt, o.data_ptr(), Wp.data_ptr(), pb.data_ptr(), M, D, D,
                               x1.data_ptr(), F32, e, st),
                epilogue(drop=d_proj.c(), resid=x2d, rowscale=rs1, rps=Nt), (x2d, rs1))
        xn2, m2, r2 = _ln(x1, n2w, n2b, dt)
        W1 = cast(f1w, dt)
        # the fc1 epilogue keeps gelu'(h) (not h) for the backward -- times the
        # dropout multiplier (FC1_FOLD) -- so the fc2 dgrad epilogue only multiplies
        # (no erf / exp, no mask hash per element);
        # with no backward to run (eval / no-grad inference) it stores gelu(h) only
        a = _empty((M, hid), dt, dev)
        if not nograd:
            gh = _empty((M, hid), dt, dev)
            _launch("vit_linear_fwd", 2.0 * M * hid * D,
                    lambda e, st=s: call("hvit_linear_fwd", dt, xn2.data_ptr(), W1.data_ptr(), f1b.data_ptr(), M, hid, D,
                                   gh.data_ptr(), dt, e, st),
                    epilogue(act=L.ACT_GELU_DUAL_DK if FC1_FOLD else L.ACT_GELU_DUAL_D, out2=a, drop=d_fc1.c()), (a,))
        else:
            gh = None
            _launch("vit_linear_fwd", 2.0 * M * hid * D,
                    lambda e, st=s: call("hvit_linear_fwd", dt, xn2.data_ptr(), W1.data_ptr(), f1b.data_ptr(), M, hid, D,
                                   a.data_ptr(), dt, e, st),
                    epilogue(act=L.ACT_GELU, drop=d_fc1.c()))
        W2 = cast(f2w, dt)
        x2 = torch.empty((M, D), dtype=torch.float32, device=dev)
        _launch("vit_linear_fwd", 2.0 * M * D * hid,
                lambda e, st=s: call("hvit_linear_fwd", dt, a.data_ptr(), W2.data_ptr(), f2b.data_ptr(), M, D, hid,
                               x2.data_ptr(), F32, e, st),
                epilogue(drop=d_fc2.c(), resid=x1, rowscale=rs2, rps=Nt), (x1, rs2))
        ctx.save_for_backward(n1w, n2w)
        ctx.wid = tuple((id(p), tuple(p.shape)) for p in (qkvw, pw, f1w, f2w))
        # the parameters whose gradients the side stream may produce (side_ok)
        ctx.prefs = tuple(weakref.ref(p) for p in (qkvw, qkvb, pw, f1w, f1b, f2w))
        ctx.wrefs = tuple(weakref.ref(p) for p in (qkvw, pw, f1w, f2w))  # (the grouped weight gradients)
        ctx.lnrefs = (weakref.ref(n1w), weakref.ref(n1b))
        ctx.kbits = kbits
        # the fc2 branch's dropout / DropPath of the incoming gradient, for the
        # next consumer of x2 to fuse into its LayerNorm backward (GradHandoff)
        if ho_out is not None and LNDROP:
            ho_out.drop, ho_out.rowscale, ho_out.rps, ho_out.dt = d_fc2.c(), rs2, Nt, dt
        ctx.ho = (ho_in if LNDROP else None, ho_out)
        ctx.t = (x2d, xn1, m1, r1, qkv, o, lse, x1, xn2, m2, r2, gh, a, Wqkv, Wp, W1, W2, rs1, rs2)
        ctx.meta = (B, Nt, D, H, hid, scale, dt, d_attn.c(), d_proj.c(), d_fc1.c(), d_fc2.c())
        # LN1, LN2 (dgamma|dbeta); fc2, proj bias grads (column sums fused into the
        # two dropout passes; fc1's comes from the GELU-backward epilogue's partial rows)
        # (LN1's / LN2's slots also hold a bias grad when a dropout pass is fused, LNDROP)
        ctx.zs = (_zs(ctx, 3 * D), _zs(ctx, 3 * D), None, _zs(ctx, D), _zs(ctx, D), _zs(ctx, 3 * D))
        if want_probs:
            ctx.mark_non_differentiable(probs)
        return x2.view(B, Nt, D), probs

    @staticmethod
    def backward(ctx, dx2, _dprobs=None):
        n1w, n2w = ctx.saved_tensors
        (x2d, xn1, m1, r1, qkv, o, lse, x1, xn2, m2, r2, gh, a, Wqkv, Wp, W1, W2, rs1, rs2) = ctx.t
        B, Nt, D, H, hid, scale, dt, dra, drp, drf1, drf2 = ctx.meta
        M = B * Nt
        dev = x1.device
        s = stream_ptr()
        dx2 = dx2.contiguous().view(M, D)
        if dx2.dtype != torch.float32:
            dx2 = dx2.float()
        # MLP branch
        zln1, zln2, _, zf2b, zpb, zqb = ctx.zs
        ho_in, ho_out = ctx.ho
        jho = None  # the consumer's deferred LN partial-row sum (GradHandoff.fuse), for a launch to carry
        if ho_out is not None and ho_out.g is not None:  # fused into the next consumer's LN backward
            g2, df2b = ho_out.g, ho_out.colsum
            if ho_out.job is not None and side_take(ho_out.job, dev):
                jho = ho_out.job
            ho_out.g = ho_out.colsum = ho_out.job = None
        else:
            g2 = _empty((M, D), dt, dev)
            df2b = zf2b.take(dev)
            dropout_scale(dx2, M, D, drf2, rs2, Nt, g2, df2b)
        dq_id, dp_id, d1_id, d2_id = ctx.wid
        # weight gradients: on the side stream, concurrent with this chain of data
        # gradients (side_ok), or else on this stream with each split-K slab sum riding
        # on the data-gradient launch that follows it (epilogue side job)
        side = side_ok(ctx.prefs)
        # or queued for one grouped launch with the other blocks' (wgrad_enqueue):
        # each then carries nothing, and the bias / LayerNorm partial-row sums the
        # weight-gradient launches carried ride on the data-gradient launches
        wq, wp, w1, w2 = ctx.wrefs
        group = (not side and wgrad_group_ok(dt, M, D, hid, w2) and wgrad_group_ok(dt, M, hid, D, w1)
                 and wgrad_group_ok(dt, M, D, D, wp) and wgrad_group_ok(dt, M, 3 * D, D, wq))

        def wdest(wid, N, K):
            d = grad_dest(*wid)
            return d if d is not None else torch.empty((N, K), dtype=torch.float32, device=dev)

        if side:
            df2w = wdest(d2_id, D, hid)
            with on_side(dev, (g2, a, df2w)):
                linear_wgrad_now(dt, g2, a, M, D, hid, dest=df2w)
            j2 = None
        elif group:
            df2w, j2 = wgrad_enqueue(g2, a, M, D, hid, grad_dest(*d2_id), w2), None
        else:
            df2w, j2 = linear_wgrad_deferred(dt, g2, a, M, D, hid, dest=grad_dest(*d2_id))
        dh = _empty((M, hid), dt, dev)
        # fc1 bias grad: the GELU-backward epilogue's column sums, one partial row per
        # 64-row block (plain stores: deterministic), summed in row order as the fc1
        # weight-gradient launch's side job
        nrow = (M + 63) // 64
        cparts = torch.empty((nrow, hid), dtype=torch.float32, device=dev)
        df1b = torch.empty(hid, dtype=torch.float32, device=dev)
        if jho is not None and j2 is not None:  # (one side job per launch)
            call("hvit_sum_slabs_strided", jho.job.src, jho.job.splits, jho.job.stride, jho.job.n, jho.job.dst, s)
            jho = None
        e_fc2 = epilogue(act=L.ACT_MUL_AUX, aux=gh, drop=None if FC1_FOLD else drf1, colsum=cparts,
                         side=j2 if j2 is not None else jho)
        _launch("vit_linear_dgrad", 2.0 * M * D * hid,
                lambda e, st=s: call("hvit_linear_dgrad", dt, g2.data_ptr(), W2.data_ptr(), M, D, hid, dh.data_ptr(), dt, e,
                               st), e_fc2, (gh, cparts))
        jc = Deferred(L.SlabSum(cparts.data_ptr(), df1b.data_ptr(), hid, hid, nrow), cparts)
        if side:
            df1w = wdest(d1_id, hid, D)
            with on_side(dev, (dh, xn2, cparts, df1b, df1w)):
                linear_wgrad_now(dt, dh, xn2, M, hid, D, dest=df1w, side=jc)
            j1 = None
        elif group:
            df1w, j1 = wgrad_enqueue(dh, xn2, M, hid, D, grad_dest(*d1_id), w1), jc
        else:
            df1w, j1 = linear_wgrad_deferred(dt, dh, xn2, M, hid, D, dest=grad_dest(*d1_id), side=jc)
        # the gradient at the LayerNorm output in the compute dtype (bf16 under the
        # bf16 model, as torch autocast's linear backward gives it): 8 MB less to
        # store and to re-read per LayerNorm backward at B=32 (dx stays f32)
        dxn2 = _empty((M, D), dt if LN_DY_LOW else F32, dev)
        e_fc1 = epilogue(side=j1)
        _launch("vit_linear_dgrad", 2.0 * M * hid * D,
                lambda e, st=s: call("hvit_linear_dgrad", dt, dh.data_ptr(), W1.data_ptr(), M, hid, D, dxn2.data_ptr(),
                               L.dt_of(dxn2),
                               e, st), e_fc1)
        jln = None
        if LNDROP:  # LN2 backward + the attention branch's dropout / DropPath scaling in one pass; its
            # [dgamma | dbeta | proj bias] partial rows summed by the proj weight-gradient launch (side job)
            dx1, dn2w, dn2b, g1, dpb, jln = _ln_bwd_drop(dxn2, x1, m2, r2, n2w, dx2, zln2, drp, rs1, Nt, dt,
                                                         defer=True)
        else:
            dx1, dn2w, dn2b = _ln_bwd(dxn2, x1, m2, r2, n2w, dx2, zln2)
            g1 = _empty((M, D), dt, dev)
            dpb = zpb.take(dev)
            dropout_scale(dx1, M, D, drp, rs1, Nt, g1, dpb)
        # attention branch
        if side:
            dpw = wdest(dp_id, D, D)
            with on_side(dev, (g1, o, dpw) + (jln.ws if jln is not None else ())):
                linear_wgrad_now(dt, g1, o, M, D, D, dest=dpw, side=jln)
            jp = None
        elif group:
            dpw, jp = wgrad_enqueue(g1, o, M, D, D, grad_dest(*dp_id), wp), jln
        else:
            dpw, jp = linear_wgrad_deferred(dt, g1, o, M, D, D, dest=grad_dest(*dp_id), side=jln)
        do = _empty((M, D), dt, dev)
        e_pr = epilogue(side=jp)
        _launch("vit_linear_dgrad", 2.0 * M * D * D,
                lambda e, st=s: call("hvit_linear_dgrad", dt, g1.data_ptr(), Wp.data_ptr(), M, D, D, do.data_ptr(), dt, e, st),
                e_pr)
        dqkv = _empty((M, 3 * D), dt, dev)
        delta = torch.empty((B, H, Nt), dtype=torch.float32, device=dev)
        # the qkv bias grad: partial column sums of dqkv written by the attention
        # backward (one row per workgroup on the register-resident kernels, one per
        # sample by a segmented column sum elsewhere; plain stores, summed in row
        # order: deterministic), summed as the qkv weight-gradient launch's side job
        jb = None
        if ATTN_DB:
            nbr = L.lib().hvit_mhsa_bias_rows(dt, B, Nt, H, D // H)
            bparts = torch.empty((nbr, 3 * D), dtype=torch.float32, device=dev)
            dqkvb = torch.empty(3 * D, dtype=torch.float32, device=dev)
            with timed("attn_bwd", 8.0 * B * H * Nt * Nt * (D // H)):
                call("hvit_mhsa_bwd_db", dt, qkv.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(), B, Nt, H,
                     D // H, scale, dra, ptr(ctx.kbits), dqkv.data_ptr(), delta.data_ptr(), bparts.data_ptr(), s)
            jb = Deferred(L.SlabSum(bparts.data_ptr(), dqkvb.data_ptr(), 3 * D, 3 * D, nbr), bparts)
        else:
            with timed("attn_bwd", 8.0 * B * H * Nt * Nt * (D // H)):
                call("hvit_mhsa_bwd_db", dt, qkv.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(), B, Nt, H,
                     D // H, scale, dra, ptr(ctx.kbits), dqkv.data_ptr(), delta.data_ptr(), None, s)
            dqkvb = zqb.take(dev)
            call("hvit_reduce_rows", dqkv.data_ptr(), dt, M, 3 * D, 3 * D, 1, dqkvb.data_ptr(), s)
        if side:
            dqkvw = wdest(dq_id, 3 * D, D)
            with on_side(dev, (dqkv, xn1, dqkvw, dqkvb) + ((jb.ws,) if jb is not None else ())):
                linear_wgrad_now(dt, dqkv, xn1, M, 3 * D, D, dest=dqkvw, side=jb)
            jq = None
        elif group:
            dqkvw, jq = wgrad_enqueue(dqkv, xn1, M, 3 * D, D, grad_dest(*dq_id), wq), jb
        else:
            dqkvw, jq = linear_wgrad_deferred(dt, dqkv, xn1, M, 3 * D, D, dest=grad_dest(*dq_id), side=jb)
        dxn1 = _empty((M, D), dt if LN_DY_LOW else F32, dev)
        e_qkv = epilogue(side=jq)
        _launch("vit_linear_dgrad", 2.0 * M * 3 * D * D,
                lambda e, st=s: call("hvit_linear_dgrad", dt, dqkv.data_ptr(), Wqkv.data_ptr(), M, 3 * D, D, dxn1.data_ptr(),
                               L.dt_of(dxn1), e, st), e_qkv)
        if ho_in is not None and ho_in.drop is not None:  # the previous block's fc2 dropout, fused
            dx, dn1w, dn1b = ho_in.fuse(dxn1, x2d, m1, r1, n1w, dx1, zln1, ctx.lnrefs)
        else:
            dx, dn1w, dn1b = _ln_bwd(dxn1, x2d, m1, r1, n1w, dx1, zln1)
        return (dx.view(B, Nt, D), dn1w, dn1b, dqkvw, dqkvb, dpw, dpb, dn2w, dn2b, df1w, df1b, df2w, df2b,
                None, None, None, None, None, None, None, None, None, None)


class HeadFn(torch.autograd.Function):
    """Final LayerNorm (attention.py:300) + to_feature_map Linear and the
    [B,N,C] -> NCHW reshape (hybrid_vit.py:342-348), which in NHWC is the
    identity: f32 tokens [B, N, D] -> NHWC feature map [B, Hp, Wp, C]."""

    @staticmethod
    def forward(ctx, x, nw, nb, w, b, hw, dt, ho: Optional[GradHandoff] = None):
        B, Nt, D = x.shape
        M = B * Nt
        C = w.shape[0]
        x2d = x.contiguous().view(M, D)
        xn, m, r = _ln(x2d, nw, nb, dt)
        W = cast(w, dt)
        y = _empty((B, hw[0], hw[1], C), dt, x.device)
        call("hvit_linear_fwd", dt, xn.data_ptr(), W.data_ptr(), b.data_ptr(), M, C, D, y.data_ptr(), dt, None,
             stream_ptr())
        ctx.save_for_backward(nw)
        ctx.t = (x2d, xn, m, r, W)
        ctx.prefs = (weakref.ref(w), weakref.ref(b))
        ctx.lnrefs = (weakref.ref(nw), weakref.ref(nb))
        ctx.meta = (B, Nt, D, C, dt)
        ctx.ho = ho if LNDROP else None
        ctx.zs = _zs(ctx, 3 * D)
        return y

    @staticmethod
    def backward(ctx, dy):
        (nw,) = ctx.saved_tensors
        x2d, xn, m, r, W = ctx.t
        B, Nt, D, C, dt = ctx.meta
        M = B * Nt
        dy = cast(dy, dt)
        dw, db, jw = _linear_wgrad_bias_maybe_side(ctx, dt, dy, xn, M, C, D)
        dxn = _empty((M, D), dt if LN_DY_LOW else F32, dy.device)
        call("hvit_linear_dgrad", dt, dy.data_ptr(), W.data_ptr(), M, C, D, dxn.data_ptr(), L.dt_of(dxn),
             epilogue(side=jw) if jw is not None else None, stream_ptr())  # (carries the wgrad's slab sum)
        if ctx.ho is not None and ctx.ho.drop is not None:  # the last block's fc2 dropout, fused
            dx, dnw, dnb = ctx.ho.fuse(dxn, x2d, m, r, nw, None, ctx.zs, ctx.lnrefs)
        else:
            dx, dnw, dnb = _ln_bwd(dxn, x2d, m, r, nw, None, ctx.zs)
        return dx.view(B, Nt, D), dnw, dnb, dw, db, None, None, None


class SkipFn(torch.autograd.Function):
    """Skip projection 1x1 conv (bias) + bilinear resize to the decoder grid
    (hybrid_vit.py:376-386).  Both are linear and the bilinear weights sum to
    one, so resize-then-project equals the reference's project-then-resize and
    the GEMM runs on the (up to 16x) smaller grid.  NHWC in / out."""

    @staticmethod
    def forward(ctx, e, w, b, Ho, Wo, dt, sg: Optional[SkipGrad] = None):
        N, He, We, Ce = e.shape
        Cd = w.shape[0]
        dev = e.device
        s = stream_ptr()
        if (He, We) != (Ho, Wo):
            r = _empty((N, Ho, Wo, Ce), dt, dev)
            call("hvit_bilinear_fwd", e.data_ptr(), dt, N, He, We, Ce, Ho, Wo, r.data_ptr(), dt, s)
        else:
            r = e.contiguous()
        W = cast(w, dt).view(Cd, Ce)
        y = _empty((N, Ho, Wo, Cd), dt, dev)
        M = N * Ho * Wo
        call("hvit_linear_fwd", dt, r.data_ptr(), W.data_ptr(), b.data_ptr(), M, Cd, Ce, y.data_ptr(), dt, None, s)
        ctx.t = (r, W)
        ctx.prefs = (weakref.ref(w), weakref.ref(b))
        ctx.meta = (N, He, We, Ce, Ho, Wo, Cd, dt, tuple(w.shape))
        ctx.sg = sg
        return y

    @staticmethod
    def backward(ctx, dy):
        r, W = ctx.t
        N, He, We, Ce, Ho, Wo, Cd, dt, wshape = ctx.meta
        M = N * Ho * Wo
        dev = r.device
        s = stream_ptr()
        dy = cast(dy, dt)
        dw, db, jw = _linear_wgrad_bias_maybe_side(ctx, dt, dy, r, M, Cd, Ce)
        dw = dw.view(wshape)
        de = None
        if jw is not None and not ctx.needs_input_grad[0]:  # no launch follows to carry the slab sum
            call("hvit_sum_slabs_strided", jw.job.src, jw.job.splits, jw.job.stride, jw.job.n, jw.job.dst, s)
        if ctx.needs_input_grad[0]:
            dr = _empty((N, Ho, Wo, Ce), dt, dev)
            call("hvit_linear_dgrad", dt, dy.data_ptr(), W.data_ptr(), M, Cd, Ce, dr.data_ptr(), dt,
                 epilogue(side=jw) if jw is not None else None, s)  # (carries the wgrad's slab sum)
            if ctx.sg is not None and ctx.sg.offer(dr, (N, Ho, Wo, Ce, He, We, dt)):
                return None, dw, db, None, None, None, None  # the encoder output's other consumer adds it
            if (He, We) != (Ho, Wo):
                de = _empty((N, He, We, Ce), dt, dev)
                call("hvit_bilinear_bwd", dr.data_ptr(), dt, N, Ho, Wo, Ce, He, We, de.data_ptr(), dt, 0, s)
            else:
                de = dr
        return de, dw, db, None, None, None, None


class FinalFn(torch.autograd.Function):
    """Final TransposeConvBlock ([up U] -> Conv -> Tanh, components.py:146-167)
    and the resize to the input size (hybrid_vit.py:459-465).  NHWC dt in,
    f32 NHWC [B, F, T, Cout] out."""

    @staticmethod
    def forward(ctx, x, w, U, out_hw, dt):
        N, Hs, Ws, C = x.shape
        Cout, Cin, KS, _ = w.shape
        H, W = Hs * U, Ws * U
        dev = x.device
        s = stream_ptr()
        wp = pack_conv(w, 0, dt)
        y = torch.empty((N, H, W, Cout), dtype=torch.float32, device=dev)
        g = geom(x, C, None, 0, N, Hs, Ws, U, KS, 1, KS // 2, Cout)
        call("hvit_conv_fwd", dt, g, wp.data_ptr(), None, y.data_ptr(), F32, None, epilogue(act=L.ACT_TANH), s)
        F, T = out_hw
        if (H, W) != (F, T):
            out = torch.empty((N, F, T, Cout), dtype=torch.float32, device=dev)
            call("hvit_bilinear_fwd", y.data_ptr(), F32, N, H, W, Cout, F, T, out.data_ptr(), F32, s)
            ctx.save_for_backward(x, w)
            ctx.y = y
        else:
            # no resize: the conv output is the result, saved as an output (autograd's version check
            # guards the tanh backward's y against in-place edits by the caller) instead of a copy
            out = y
            ctx.save_for_backward(x, w, out)
            ctx.y = None
        ctx.meta = (U, out_hw, dt)
        return out

    @staticmethod
    def backward(ctx, dout):
        saved = ctx.saved_tensors
        x, w = saved[0], saved[1]
        U, (F, T), dt = ctx.meta
        y = ctx.y if ctx.y is not None else saved[2]
        N, H, W, Cout = y.shape
        Hs, Ws, C = x.shape[1], x.shape[2], x.shape[3]
        KS = w.shape[2]
        dev = x.device
        s = stream_ptr()
        dout = dout.contiguous().float()
        if (H, W) != (F, T):
            dy = torch.empty((N, H, W, Cout), dtype=torch.float32, device=dev)
            call("hvit_bilinear_bwd", dout.data_ptr(), F32, N, F, T, Cout, H, W, dy.data_ptr(), F32, 0, s)
        else:
            dy = dout
        dz = _empty((N, H, W, Cout), dt, dev)
        call("hvit_tanh_bwd", dy.data_ptr(), F32, y.data_ptr(), dy.numel(), dz.data_ptr(), dt, s)
        g = geom(x, C, None, 0, N, Hs, Ws, U, KS, 1, KS // 2, Cout)
        dw = conv_wgrad(dt, g, dz, w.shape)
        dx = None
        if ctx.needs_input_grad[0]:
            wd = pack_conv(w, 1, dt)
            du = _empty((N, H, W, C), dt, dev)
            call("hvit_conv_dgrad", dt, g, dz.data_ptr(), wd.data_ptr(), du.data_ptr(), dt, s)
            if U == 1:
                dx = du
            else:
                dx = _empty((N, Hs, Ws, C), dt, dev)
                call("hvit_upsample_split_bwd", du.data_ptr(), dt, N, Hs, Ws, U, C, 0, dx.data_ptr(), dt, None, dt, s)
        return dx, dw, None, None, None
