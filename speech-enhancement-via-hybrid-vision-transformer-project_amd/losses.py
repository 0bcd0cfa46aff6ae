"""CombinedLoss (training/losses.py:286-408 of the reference), the loss on the
timed training step of BASELINE config 3.

Same weights and semantics: l1_weight * L1 + mse_weight * MSE + stoi_weight *
mean(1 - cos(flatten(pred), flatten(target))) (+ perceptual = L1).  Unlike the
reference it does not call ``.item()`` on every component (losses.py:362-383,
four device->host syncs per step); ``return_components=True`` still returns the
per-component values, as tensors.
"""

from __future__ import annotations

from typing import Dict

import torch
import torch.nn as nn
import torch.nn.functional as F


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
        pred = pred.float()
        target = target.float()
        pi, ti = pred, target
        if self.use_log_compression:
            pi, ti = torch.log(pred + 1e-8), torch.log(target + 1e-8)
        comps = {}
        total = pred.new_zeros(())
        if self.l1_weight > 0:
            comps["l1"] = F.l1_loss(pi, ti)
            total = total + self.l1_weight * comps["l1"]
        if self.mse_weight > 0:
            comps["mse"] = F.mse_loss(pi, ti)
            total = total + self.mse_weight * comps["mse"]
        if self.stoi_weight > 0:
            pn = F.normalize(pred.flatten(1), dim=1)
            tn = F.normalize(target.flatten(1), dim=1)
            comps["stoi"] = (1.0 - (pn * tn).sum(1)).mean()
            total = total + self.stoi_weight * comps["stoi"]
        if self.perceptual_weight > 0:
            comps["perceptual"] = F.l1_loss(pred, target)
            total = total + self.perceptual_weight * comps["perceptual"]
        comps["total"] = total
        if return_components:
            return total, comps
        return total


def create_loss_function(config: Dict) -> nn.Module:
    """losses.py:390-408."""
    lc = config.get("loss", {})
    return CombinedLoss(l1_weight=lc.get("l1_weight", 1.0), mse_weight=lc.get("mse_weight", 0.0),
                        stoi_weight=lc.get("stoi_weight", 0.1), perceptual_weight=lc.get("perceptual_weight", 0.0),
                        use_log_compression=lc.get("use_log_compression", False))
