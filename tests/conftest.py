import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def hv():
    import hvit_amd_loader

    return hvit_amd_loader.load()


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


# --- numpy mirror of the counter-based dropout hash (csrc/common.h) ----------
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _hash32(x):
    """lowbias32 on uint32 arrays (csrc/common.h hash32)."""
    x = x.astype(np.uint32)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x7FEB352D)
        x ^= x >> np.uint32(15)
        x *= np.uint32(0x846CA68B)
        x ^= x >> np.uint32(16)
    return x


def rng_key(seed, site):
    m = int(_mix64(np.uint64(seed) ^ (np.uint64(site) << np.uint64(48))))
    return np.uint32((m ^ (m >> 32)) & 0xFFFFFFFF)


def keep_mask(seed, site, n, p):
    """Boolean keep mask for element indices 0..n-1 (same as rng_keep):
    one lowbias32 hash per element pair, 16 bits per element."""
    idx = np.arange(n, dtype=np.uint64)
    pair = (idx >> np.uint64(1)).astype(np.uint32)  # 32-bit pair counter (wraps past 2^33)
    h = _hash32(rng_key(seed, site) ^ pair)
    u16 = (h >> (np.uint32(16) * (idx & np.uint64(1)).astype(np.uint32))) & np.uint32(0xFFFF)
    thr = 0 if p <= 0 else min(65536, int(p * 65536.0 + 0.5))
    return u16 >= np.uint32(thr)
