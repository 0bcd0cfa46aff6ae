"""CPU: the C-ABI library loads and exports every symbol include/hvit.h
declares; the drop-in module reproduces the reference's constructor surface,
state_dict keys/shapes, parameter counts and factory; the HIP path refuses to
run on CPU tensors (no silent fallback)."""

import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import closed_form as CF
from oracle import hvit_oracle as O

HEADER = os.path.join(ROOT, "include", "hvit.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hvit_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(hv):
    lib = hv._lib.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(hv._lib.EXPORTED), set(syms) ^ set(hv._lib.EXPORTED)
    assert lib.hvit_version().decode().startswith("hvit")


def test_error_reporting_without_gpu_work(hv):
    L = hv._lib
    # invalid arguments are rejected on the host before any launch
    with pytest.raises(RuntimeError, match="null pointer"):
        L.call("hvit_linear_fwd", L.F32, None, None, None, 4, 4, 4, None, L.F32, None, None)
    with pytest.raises(RuntimeError, match="head_dim"):
        L.call("hvit_mhsa_fwd", L.F32, 16, 1, 4, 1, 48, 0.1, None, 16, 16, None, None)


def test_wgrad_workspace_query(hv):
    n = hv._lib.lib().hvit_wgrad_workspace(8192, 512, 512)
    # whole split-K slabs, each dw [N, K] followed by the N bias partials
    assert n >= 0 and n % (512 * 512 + 512) == 0


@pytest.mark.parametrize("kw", [{}, O.TINY, dict(num_layers=12, num_heads=12, embed_dim=768),
                                dict(O.TINY, use_cls_token=True)])
def test_state_dict_matches_reference(hv, kw):
    m = hv.HybridViT(**kw)
    shapes = O.state_dict_shapes(O.HViTConfig(**kw))
    sd = m.state_dict()
    assert list(sd.keys()) == list(shapes.keys())
    for k, v in sd.items():
        assert tuple(v.shape) == shapes[k], k
    if not kw:
        assert len(sd) == 122
        assert m.count_parameters()["total"] == 28454976


def test_load_reference_weights_strict(hv):
    cfg = O.HViTConfig(**O.TINY)
    W = CF.weights(O.state_dict_shapes(cfg))
    m = hv.HybridViT(**cfg.as_kwargs())
    m.load_state_dict({k: torch.as_tensor(v) for k, v in W.items()}, strict=True)
    assert torch.equal(m.encoder[0].block[0].weight, torch.as_tensor(W["encoder.0.block.0.weight"]))


def test_create_hybrid_vit_config_keys(hv):
    cfg = {"model": {"encoder": {"channels": [8, 16, 32], "dropout": 0.2},
                     "transformer": {"embed_dim": 64, "num_heads": 4, "num_layers": 2, "attention_dropout": 0.05,
                                     "drop_path_rate": 0.0},
                     "decoder": {"channels": [32, 16, 8, 1]}}}
    m = hv.create_hybrid_vit(cfg)
    assert m.embed_dim == 64 and len(m.transformer.blocks) == 2
    assert m.encoder[0].p == 0.2 and m.transformer.blocks[0].p_attn == 0.05
    assert hv.create_hybrid_vit().count_parameters()["total"] == 28454976


def test_init_matches_reference_statistics(hv):
    torch.manual_seed(0)
    m = hv.HybridViT(**O.TINY)
    w = m.transformer.blocks[0].attn.qkv.weight
    # trunc_normal_(std=0.02) with torch's default absolute bounds [-2, 2] (as the reference calls it)
    assert abs(w.std().item() - 0.02) < 0.003 and w.abs().max().item() < 0.2
    assert torch.all(m.transformer.blocks[0].attn.qkv.bias == 0)
    assert torch.all(m.encoder[0].block[1].weight == 1)
    assert abs(m.pos_encoding.pos_embed.std().item() - 0.02) < 0.003


def test_cpu_tensor_is_refused(hv):
    m = hv.HybridViT(**O.TINY)
    with pytest.raises(RuntimeError, match="GPU"):
        m(torch.zeros(1, 1, 32, 32))


def test_dropout_mask_mirror_statistics():
    from conftest import keep_mask

    k = keep_mask(1234, 7, 1 << 16, 0.1)
    assert abs(1.0 - k.mean() - 0.1) < 0.01
    assert not np.array_equal(k, keep_mask(1235, 7, 1 << 16, 0.1))
