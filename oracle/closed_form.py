"""Deterministic, platform-independent parameter/input generator for parity tests.

TEST INFRASTRUCTURE ONLY (see oracle/hvit_oracle.py header).

The default-config golden vectors cannot commit 28 M weights, so every fixture is
defined over weights produced here from numpy's PCG64 stream (stable across
platforms and numpy versions for ``Generator.random``).  The GPU box regenerates
the same weights without torch RNG or the reference.  Scales follow fan-in so
activations stay O(1); BN running statistics are non-trivial so eval-mode BN is
exercised; the final decoder conv is damped so tanh does not saturate (a
saturated output makes output parity vacuous, SURVEY §7 hard part 4).
"""

from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np


def _u(seed: int, n: int) -> np.ndarray:
    return np.random.Generator(np.random.PCG64(seed)).random(n)


def weights(shapes: Dict[str, Tuple[int, ...]], seed: int = 20240601) -> Dict[str, np.ndarray]:
    out: Dict[str, np.ndarray] = {}
    keys = list(shapes)
    final_conv = [k for k in keys if k.startswith("decoder.") and k.endswith(".weight")
                  and len(shapes[k]) == 4][-1]
    for t, k in enumerate(keys):
        shp = shapes[k]
        if k.endswith("num_batches_tracked"):
            out[k] = np.zeros((), np.int64)
            continue
        n = int(np.prod(shp)) if len(shp) else 1
        s = 2.0 * _u(seed + 7919 * t, n) - 1.0          # U(-1, 1)
        if k.endswith("running_mean"):
            v = 0.1 * s
        elif k.endswith("running_var"):
            v = 1.0 + 0.5 * s
        elif "pos_embed" in k or k == "cls_token":
            v = 0.035 * s
        elif len(shp) == 4:                              # conv weights
            fan_in = shp[1] * shp[2] * shp[3]
            gain = 2.0 if (k.startswith("encoder") or k.startswith("decoder")) else 1.0
            v = s * math.sqrt(3.0 * gain / fan_in)
            if k == final_conv:
                v = v * 0.5
        elif len(shp) == 2:                              # linear weights
            v = s * math.sqrt(3.0 / shp[1])
        elif k.endswith(".weight"):                      # BN / LN gamma
            v = 1.0 + 0.2 * s
        else:                                            # biases, BN/LN beta
            v = 0.05 * s
        out[k] = v.astype(np.float32).reshape(shp)
    return out


def spectrogram(shape, seed: int) -> np.ndarray:
    """Input magnitudes in [0, 1) (the range of a per-utterance min-max
    normalised spectrogram, data/dataset.py:213-219)."""
    return _u(seed, int(np.prod(shape))).astype(np.float32).reshape(shape)
