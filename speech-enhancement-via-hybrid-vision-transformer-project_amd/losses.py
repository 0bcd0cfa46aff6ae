"""CombinedLoss (training/losses.py:286-408 of the reference), the loss on the
timed training step of BASELINE config 3, on libhvit.so.

Same weights and semantics: l1_weight * L1 + mse_weight * MSE + stoi_weight *
mean_b(1 - cos(flatten(pred_b), flatten(target_b))) (STOILoss :109-141) +
perceptual_weight * L1 (PerceptualLoss :270-283), L1/MSE on log(x + 1e-8)
when ``use_log_compression`` (:319-321).  One pass over pred/target
(hvit_loss_fwd) yields the loss, its components and the per-sample sums the
backward (hvit_loss_bwd) needs.  Unlike the reference it does not call
``.item()`` on every component (losses.py:362-383, four device->host syncs per
step); ``return_components=True`` returns the components as 0-dim tensors.
"""

from __future__ import annotations

from typing import Dict

import torch
import torch.nn as nn

from . import _lib as L


class CombinedLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, cfg: "L.LossCfg"):
        B = pred.shape[0]
        P = pred.numel() // max(B, 1)
        dev = pred.device
        ws_n = L.lib().hvit_loss_ws_elems(B, P)
        ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=dev)
        stats = torch.empty((B, 6), dtype=torch.float32, device=dev)
        out = torch.empty(5, dtype=torch.float32, device=dev)
        L.call("hvit_loss_fwd", pred.data_ptr(), target.data_ptr(), B, P, cfg, ws.data_ptr(), ws_n,
               stats.data_ptr(), out.data_ptr(), L.stream_ptr())
        ctx.save_for_backward(pred, target, stats)
        ctx.cfg = cfg
        comps = out[1:]
        ctx.mark_non_differentiable(comps)
        ctx.set_materialize_grads(False)  # (no zero-filled gradient for the components: one launch fewer)
        return out[0], comps

    @staticmethod
    def backward(ctx, gtot, _gcomps=None):
        if gtot is None:
            return None, None, None
        pred, target, stats = ctx.saved_tensors
        B = pred.shape[0]
        P = pred.numel() // B
        g = gtot.detach().float().contiguous()
        dpred = torch.empty_like(pred)
        L.call("hvit_loss_bwd", pred.data_ptr(), target.data_ptr(), B, P, ctx.cfg, stats.data_ptr(), g.data_ptr(),
               dpred.data_ptr(), L.stream_ptr())
        return dpred, None, None


class CombinedLoss(nn.Module):
    def __init__(self, l1_weight: float = 1.0, mse_weight: float = 0.0, stoi_weight: float = 0.1,
                 perceptual_weight: float = 0.0, use_log_compression: bool = False):
        super().__init__()
        self.l1_weight = l1_weight
        self.mse_weight = mse_weight
        self.stoi_weight = stoi_weight
        self.perceptual_weight = perceptual_weight
        self.use_log_compression = use_log_compression

    def forward(self, pred, target, return_components: bool = False):
        if not pred.is_cuda or not target.is_cuda:
            raise RuntimeError("hvit CombinedLoss: the HIP path needs GPU tensors; there is no CPU path")
        if target.requires_grad:
            raise NotImplementedError("hvit CombinedLoss: gradients w.r.t. the target are not supported")
        if pred.shape != target.shape or pred.dim() < 2 or pred.shape[0] == 0:
            raise ValueError(f"hvit CombinedLoss: shape mismatch {tuple(pred.shape)} vs {tuple(target.shape)}")
        p = pred.float().contiguous()
        t = target.detach().float().contiguous()
        cfg = L.LossCfg(self.l1_weight, self.mse_weight, self.stoi_weight, self.perceptual_weight,
                        int(bool(self.use_log_compression)))
        total, comps = CombinedLossFn.apply(p, t, cfg)
        if not return_components:
            return total
        names = ("l1", "mse", "stoi", "perceptual")
        weights = (self.l1_weight, self.mse_weight, self.stoi_weight, self.perceptual_weight)
        out = {n: comps[i] for i, (n, w) in enumerate(zip(names, weights)) if w > 0}
        out["total"] = total.detach()
        return total, out


def create_loss_function(config: Dict) -> nn.Module:
    """losses.py:390-408."""
    lc = config.get("loss", {})
    return CombinedLoss(l1_weight=lc.get("l1_weight", 1.0), mse_weight=lc.get("mse_weight", 0.0),
                        stoi_weight=lc.get("stoi_weight", 0.1), perceptual_weight=lc.get("perceptual_weight", 0.0),
                        use_log_compression=lc.get("use_log_compression", False))
