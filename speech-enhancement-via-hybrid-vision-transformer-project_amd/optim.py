"""AdamW and gradient clipping of the reference training step on libhvit.so.

The reference trainer builds ``torch.optim.AdamW(model.parameters(), lr,
betas, eps, weight_decay, amsgrad)`` in ``create_optimizer``
(training/optimizer.py:20-73, AdamW :53-61) and clips with
``torch.nn.utils.clip_grad_norm_(model.parameters(), max_grad_norm)``
(training/trainer.py:170-174).  Here:

* ``clip_grad_norm_`` -- same signature and in-place semantics (2-norm):
  one multi-tensor sum-of-squares launch + one finalize block + one scale
  launch, no host sync; returns the total norm as a 0-dim device tensor.
* ``FusedAdamW`` -- torch.optim.AdamW's update rule (decoupled weight decay,
  bias corrections, per-parameter ``step``) as multi-tensor launches of at
  most 60 tensors each, balanced (HybridViT's 104: two of 52).  With ``max_grad_norm`` the clip is fused: the update multiplies
  each gradient by the clip coefficient as it reads it (gradients are not
  rewritten; ``last_grad_norm`` holds the norm).  It also writes the bf16 copy
  of each updated linear weight that the next bf16 forward's GEMMs read
  (functional.shadow_*), so that forward skips the per-step weight cast.
* ``create_optimizer`` -- the reference factory, returning FusedAdamW for
  'adamw' and the torch optimizers for 'adam' / 'sgd'.
"""

from __future__ import annotations

from typing import Any, Dict, Optional

import torch

from . import _lib as L
from . import functional as HF

_bump = getattr(torch.autograd.graph, "increment_version", None)


def _grads(parameters) -> list:
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    return [p.grad for p in parameters if p.grad is not None]


def _refs(tensors) -> "L.TensorRef * n":
    arr = (L.TensorRef * max(len(tensors), 1))()
    for i, t in enumerate(tensors):
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise TypeError("hvit: gradients must be contiguous float32 GPU tensors")
        arr[i] = L.TensorRef(t.data_ptr(), t.numel())
    return arr


def _clip_coef(grads, max_norm: float) -> torch.Tensor:
    """[norm, min(max_norm / (norm + 1e-6), 1)] on the device."""
    dev = grads[0].device
    out = torch.empty(2, dtype=torch.float32, device=dev)
    ws_n = L.lib().hvit_clip_ws_elems(len(grads))
    ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=dev)
    L.call("hvit_clip_coef", len(grads), _refs(grads), float(max_norm), ws.data_ptr(), ws_n, out.data_ptr(),
           L.stream_ptr(dev))
    return out


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0, error_if_nonfinite: bool = False,
                    foreach=None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ (as called at trainer.py:171-174) for the
    2-norm: grads *= min(max_norm / (total_norm + 1e-6), 1) in place."""
    if float(norm_type) != 2.0:
        raise NotImplementedError("hvit clip_grad_norm_: only the 2-norm (the trainer's) is implemented")
    grads = _grads(parameters)
    if not grads:
        return torch.tensor(0.0)
    out = _clip_coef(grads, max_norm)
    if error_if_nonfinite and not torch.isfinite(out[0]).item():
        raise RuntimeError("hvit clip_grad_norm_: the total norm of the gradients is non-finite")
    L.call("hvit_scale_tensors", len(grads), _refs(grads), out.data_ptr(), L.stream_ptr(grads[0].device))
    return out[0]


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW (amsgrad=False, maximize=False) on libhvit.so, with
    optional fused gradient clipping (``max_grad_norm``)."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, amsgrad: bool = False, *, maximize: bool = False,
                 max_grad_norm: Optional[float] = None, capturable: bool = False, **unused):
        if amsgrad or maximize:
            raise NotImplementedError("hvit FusedAdamW: amsgrad / maximize are not implemented")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError("hvit FusedAdamW: invalid hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False))
        self.max_grad_norm = max_grad_norm
        self.last_grad_norm: Optional[torch.Tensor] = None
        # capturable (torch.optim.AdamW's flag): step counters live on the device
        # (0-dim views of one buffer per group, bumped by one launch) and the bias
        # corrections are computed there, so a captured step (hipGraph) replays
        # with the right step count; otherwise CPU counters as torch's default
        self.capturable = capturable
        self._step_bufs: Dict[int, torch.Tensor] = {}
        # capturable: each group's [lr, beta1, beta2, eps, weight_decay] also live
        # on the device and the kernel reads them there, so a captured step
        # replays the values of the latest sync_hyper() (an LR scheduler's), not
        # the ones it was captured with (GraphedTrainStep syncs before a replay)
        self._hyper_bufs: Dict[int, torch.Tensor] = {}
        self._hyper_vals: Dict[int, tuple] = {}

    @staticmethod
    def _hyper_of(group) -> tuple:
        b1, b2 = group["betas"]
        return (float(group["lr"]), float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]))

    def sync_hyper(self) -> None:
        """Write every group's current hyper-parameters to its device buffer
        (stream-ordered; only when they changed).  Not during stream capture:
        a captured copy would replay the capture-time values."""
        if not self.capturable or torch.cuda.is_current_stream_capturing():
            return
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.requires_grad]
            if not ps or not ps[0].is_cuda:
                continue
            vals = self._hyper_of(group)
            buf = self._hyper_bufs.get(gi)
            if buf is None or buf.device != ps[0].device:
                buf = self._hyper_bufs[gi] = torch.empty(5, dtype=torch.float32, device=ps[0].device)
                self._hyper_vals.pop(gi, None)
            if self._hyper_vals.get(gi) != vals:
                buf.copy_(torch.tensor(vals, dtype=torch.float32).pin_memory(), non_blocking=True)
                self._hyper_vals[gi] = vals

    def _device_steps(self, gi: int, ps: list) -> torch.Tensor:
        """The group's device step buffer, state["step"] of every parameter a
        0-dim view of it (rebuilt eagerly from the current values when the
        views were replaced, e.g. by load_state_dict)."""
        buf = self._step_bufs.get(gi)
        ok = buf is not None and buf.numel() == len(ps) and buf.device == ps[0].device
        if ok:
            base = buf.data_ptr()
            ok = all(isinstance(self.state[p].get("step"), torch.Tensor) and self.state[p]["step"].data_ptr() == base + 4 * i
                     for i, p in enumerate(ps))
        if not ok:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("hvit FusedAdamW(capturable=True): run one eager step before capturing")
            vals = [float(self.state[p]["step"]) if "step" in self.state[p] else 0.0 for p in ps]
            buf = torch.tensor(vals, dtype=torch.float32).to(ps[0].device)
            self._step_bufs[gi] = buf
            for i, p in enumerate(ps):
                self.state[p]["step"] = buf[i]
        return buf

    def state_dict(self):
        """torch.optim.AdamW's format.  With ``capturable`` every parameter that
        requires grad gets a device step view, including ones that never had a
        gradient; such step-only entries (no ``exp_avg`` / ``exp_avg_sq``) are
        dropped, so the dict loads into torch.optim.AdamW (whose step raises a
        KeyError on a non-empty state without the moments)."""
        sd = super().state_dict()
        sd["state"] = {k: v for k, v in sd["state"].items() if "exp_avg" in v}
        return sd

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        live = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
        if not live:
            return loss
        for p in live:
            if p.grad.is_sparse:
                raise RuntimeError("hvit FusedAdamW: sparse gradients are not supported")
            if not p.is_cuda or p.dtype != torch.float32:
                raise TypeError("hvit FusedAdamW: parameters must be float32 GPU tensors")
            # the kernel walks p, grad, exp_avg and exp_avg_sq as flat arrays: all
            # four must share one dense layout (a channels_last parameter with a
            # contiguous grad would pair the wrong elements)
            if not p.is_contiguous() or not p.grad.is_contiguous():
                raise ValueError("hvit FusedAdamW: parameters and their gradients must be contiguous "
                                 "(a strided / channels_last parameter is not supported)")
        coef = None
        if self.max_grad_norm is not None:
            coef = _clip_coef([p.grad for p in live], self.max_grad_norm)
            self.last_grad_norm = coef[0]
        stream = L.stream_ptr(live[0].device)
        if self.capturable:
            self.sync_hyper()
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            by_step: Dict[float, list] = {}
            ps_live = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if "exp_avg" not in st:
                    st.setdefault("step", torch.tensor(0.0))
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                ps_live.append(p)
            if self.capturable:
                # device counters: one bump launch, bias corrections on the device
                gp = [p for p in group["params"] if p.requires_grad]
                buf = self._device_steps(gi, gp)
                if len(ps_live) == len(gp):
                    L.call("hvit_step_bump", buf.data_ptr(), buf.numel(), 1.0, stream)
                else:
                    for p in ps_live:
                        L.call("hvit_step_bump", self.state[p]["step"].data_ptr(), 1, 1.0, stream)
                by_step = {None: ps_live} if ps_live else {}
            else:
                # per-parameter step counters stay CPU tensors (torch.optim.AdamW's
                # state_dict format); one multi-tensor add instead of one op each
                steps = [self.state[p]["step"] for p in ps_live]
                if steps:
                    torch._foreach_add_(steps, 1.0)
                for p, t in zip(ps_live, steps):
                    by_step.setdefault(t.item(), []).append(p)
            for step, ps in by_step.items():
                items = (L.AdamWItem * len(ps))()
                for i, p in enumerate(ps):
                    st = self.state[p]
                    g = p.grad
                    sh = HF.shadow_of(p)
                    items[i] = L.AdamWItem(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                           st["exp_avg_sq"].data_ptr(), sh.data_ptr() if sh is not None else None,
                                           p.numel(), st["step"].data_ptr() if step is None else None)
                bc1, bc2 = (1.0, 1.0) if step is None else (1.0 - b1 ** step, 1.0 - b2 ** step)
                hp = L.AdamWHyper(float(group["lr"]), b1, b2, group["eps"], group["weight_decay"], bc1, bc2)
                # read p, g, m, v f32, write p, m, v f32 (+ the bf16 shadow)
                nbytes = (float(sum(p.numel() * (28 + (2 if HF.shadow_of(p) is not None else 0)) for p in ps))
                          if HF.OP_TIMES is not None else 0.0)
                hbuf = self._hyper_bufs.get(gi) if self.capturable else None
                if self.capturable and hbuf is None:
                    raise RuntimeError("hvit FusedAdamW(capturable=True): run one eager step before capturing")
                with HF.timed("adamw", nbytes):
                    L.call("hvit_adamw_dev", len(ps), items, hp, coef.data_ptr() if coef is not None else None,
                           hbuf.data_ptr() if hbuf is not None else None, stream)
                for p in ps:
                    if _bump is not None:
                        _bump(p)  # the kernel wrote p in place: keep version counters honest
                    HF.shadow_mark(p)
        # parameters changed: no inference forward may reuse a packed / BN-folded
        # copy (a captured replay of this step bumps no version counter)
        HF.prep_cache_clear()
        return loss


def create_optimizer(model: torch.nn.Module, config: Dict[str, Any]) -> torch.optim.Optimizer:
    """training/optimizer.py:20-73 with AdamW on the HIP path."""
    oc = config.get("optimizer", {})
    name = oc.get("name", "adamw").lower()
    lr = oc.get("lr", 1e-4)
    wd = oc.get("weight_decay", 0.01)
    if name == "adamw":
        return FusedAdamW(model.parameters(), lr=lr, betas=oc.get("betas", (0.9, 0.999)), eps=oc.get("eps", 1e-8),
                          weight_decay=wd, amsgrad=oc.get("amsgrad", False))
    if name == "adam":
        return torch.optim.Adam(model.parameters(), lr=lr, betas=oc.get("betas", (0.9, 0.999)),
                                eps=oc.get("eps", 1e-8), weight_decay=wd, amsgrad=oc.get("amsgrad", False))
    if name == "sgd":
        return torch.optim.SGD(model.parameters(), lr=lr, momentum=oc.get("momentum", 0.9), weight_decay=wd,
                               nesterov=oc.get("nesterov", True))
    raise ValueError(f"Unknown optimizer: {name}")
