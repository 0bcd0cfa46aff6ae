"""GPU: BASELINE config 1 plumbing -- a synthetic 2 s clip through the
enhancer (host STFT, HybridViT on the HIP path, host iSTFT) against the same
enhancer around the CPU oracle forward."""

import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import closed_form as CF
from oracle import hvit_oracle as O

pytestmark = pytest.mark.gpu


class OracleModel(nn.Module):
    def __init__(self, sd, cfg):
        super().__init__()
        self.sd, self.cfg = sd, cfg

    def forward(self, x):
        return O.forward(self.sd, x.cpu(), self.cfg, training=False)


def test_enhance_clip_matches_oracle(hv):
    from hvit_amd import enhancer as E

    cfg = O.HViTConfig(**O.TINY)
    shapes = O.state_dict_shapes(cfg)
    W = CF.weights(shapes)
    m = hv.HybridViT(**cfg.as_kwargs(), precision="fp32")
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    clip = E.synthetic_clip(2.0, seed=5)
    out = E.AudioEnhancer(m, device="cuda").enhance(clip)
    ref = E.AudioEnhancer(OracleModel(O.make_state(shapes, W), cfg), device="cpu").enhance(clip)
    assert out.shape == clip.shape
    assert np.abs(out - ref).max() < 2e-3 * np.abs(ref).max()
