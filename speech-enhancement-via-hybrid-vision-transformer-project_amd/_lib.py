"""ctypes binding of libhvit.so (the C ABI declared in include/hvit.h).

The library is built in-tree by ``__graft_entry__.build()`` (csrc/Makefile) and
loaded from this directory.  There is no fallback: if the library is missing or
a call fails, a RuntimeError is raised with the library's error message.
"""

from __future__ import annotations

import ctypes as C
import os
import threading

import torch

F32, BF16 = 0, 1
ACT_NONE, ACT_GELU_DUAL, ACT_TANH, ACT_GELU_BWD, ACT_GELU_DUAL_D, ACT_MUL_AUX, ACT_RELU, ACT_GELU, ACT_RELU_POOL2 = (
    0, 1, 2, 3, 4, 5, 6, 7, 8)
ACT_GELU_DUAL_DK = 9
ACC_ZEROED = 1
ACC_DEFER = 2

_HERE = os.path.dirname(os.path.abspath(__file__))
# HVIT_LIB selects an alternative in-tree build (kernel A/B benchmarking only)
LIB_PATH = os.path.join(_HERE, os.environ.get("HVIT_LIB", "libhvit.so"))

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_longlong
f32 = C.c_float


class Dropout(C.Structure):
    _fields_ = [("p", C.c_float), ("seed", C.c_ulonglong), ("site", C.c_uint), ("seed_ptr", C.c_void_p)]


class SlabSum(C.Structure):
    """hvit_slab_sum_t: split-K slabs of a deferred weight gradient."""
    _fields_ = [("src", vp), ("dst", vp), ("n", i64), ("stride", i64), ("splits", i32)]


class WgradProb(C.Structure):
    """hvit_wgrad_prob_t: one weight gradient of a grouped launch."""
    _fields_ = [("dy", vp), ("ldy", i32), ("x", vp), ("ldx", i32), ("dw", vp), ("n_out", i32), ("k_in", i32),
                ("patch", i32), ("img_h", i32), ("img_w", i32), ("img_c", i32)]


class Epilogue(C.Structure):
    _fields_ = [
        ("act", i32), ("out2", vp), ("out2_dt", i32), ("aux", vp), ("aux_dt", i32),
        ("dropout", Dropout), ("resid", vp), ("rowscale", vp), ("rows_per_sample", i32),
        ("rowadd", vp), ("rowadd_rows", i32), ("colsum", vp), ("side", SlabSum),
    ]


class ConvGeom(C.Structure):
    _fields_ = [
        ("src1", vp), ("C1", i32), ("src2", vp), ("C2", i32),
        ("N", i32), ("Hs", i32), ("Ws", i32), ("U", i32),
        ("KS", i32), ("stride", i32), ("pad", i32), ("Cout", i32),
    ]


class WPrepItem(C.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("numel", i64), ("kind", i32), ("dt", i32),
                ("cout", i32), ("cin", i32), ("ks", i32), ("gamma", vp), ("beta", vp), ("rmean", vp),
                ("rvar", vp), ("bias", vp), ("eps", f32)]


class LossCfg(C.Structure):
    _fields_ = [("w_l1", f32), ("w_mse", f32), ("w_stoi", f32), ("w_perc", f32), ("log_compression", i32)]


class TensorRef(C.Structure):
    _fields_ = [("ptr", vp), ("numel", i64)]


class AdamWItem(C.Structure):
    _fields_ = [("param", vp), ("grad", vp), ("exp_avg", vp), ("exp_avg_sq", vp), ("shadow_bf16", vp),
                ("numel", i64), ("step", vp)]


class AdamWHyper(C.Structure):
    _fields_ = [("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("weight_decay", f32), ("bc1", f32),
                ("bc2", f32)]


P = C.POINTER
_SIGS = {
    "hvit_last_error": ([], C.c_char_p),
    "hvit_version": ([], C.c_char_p),
    "hvit_linear_fwd": ([i32, vp, vp, vp, i32, i32, i32, vp, i32, P(Epilogue), vp], i32),
    "hvit_linear_dgrad": ([i32, vp, vp, i32, i32, i32, vp, i32, P(Epilogue), vp], i32),
    "hvit_wgrad_workspace": ([i32, i32, i32], i64),
    "hvit_linear_wgrad": ([i32, vp, vp, i32, i32, i32, vp, vp, vp, i64, vp], i32),
    "hvit_wgrad_tickets": ([i32, i32, i32], i64),
    "hvit_linear_wgrad_defer": ([i32, vp, vp, i32, i32, i32, vp, vp, i64, P(SlabSum), P(SlabSum), vp], i32),
    "hvit_linear_wgrad_bias_defer": ([i32, vp, vp, i32, i32, i32, vp, vp, vp, i64, P(SlabSum), P(SlabSum), vp],
                                     i32),
    "hvit_mhsa_bias_rows": ([i32, i32, i32, i32, i32], i64),
    "hvit_sum_slabs_strided": ([vp, i32, i64, i64, vp, vp], i32),
    "hvit_linear_wgrad_group_ok": ([i32, i32, i32, i32], i32),
    "hvit_linear_wgrad_group_patch_ok": ([i32, i32, i32, i32, i32, i32, i32], i32),
    "hvit_linear_wgrad_group_ws": ([], i64),
    "hvit_linear_wgrad_group_tickets": ([], i64),
    "hvit_linear_wgrad_group": ([i32, i32, P(WgradProb), i32, vp, i64, vp, i64, vp], i32),
    "hvit_linear_wgrad_tk": ([i32, vp, vp, i32, i32, i32, vp, vp, vp, i64, vp, i64, i32, vp], i32),
    "hvit_conv_fwd": ([i32, P(ConvGeom), vp, vp, vp, i32, vp, P(Epilogue), vp], i32),
    "hvit_conv_dgrad": ([i32, P(ConvGeom), vp, vp, vp, i32, vp], i32),
    "hvit_conv_wgrad_workspace": ([P(ConvGeom)], i64),
    "hvit_conv_wgrad": ([i32, P(ConvGeom), vp, vp, vp, i64, vp], i32),
    "hvit_conv_wgrad_torch": ([i32, P(ConvGeom), vp, vp, vp, vp, i64, vp], i32),
    "hvit_conv_weight_pack": ([vp, i32, i32, i32, i32, vp, i32, vp], i32),
    "hvit_conv_weight_unpack": ([vp, i32, i32, i32, vp, vp], i32),
    "hvit_bn_fold": ([vp, i32, i32, i32, vp, vp, vp, vp, vp, i32, vp, vp], i32),
    "hvit_mhsa_fwd": ([i32, vp, i32, i32, i32, i32, f32, P(Dropout), vp, vp, vp, vp], i32),
    "hvit_mhsa_fwd_fp8": ([vp, i32, i32, i32, i32, f32, P(Dropout), vp, vp, vp], i32),
    "hvit_mhsa_fwd_fp8_kb": ([vp, i32, i32, i32, i32, f32, P(Dropout), vp, vp, vp, vp], i32),
    "hvit_mhsa_bwd": ([i32, vp, vp, vp, vp, i32, i32, i32, i32, f32, P(Dropout), vp, vp, vp], i32),
    "hvit_mhsa_keep_bits_elems": ([i32, i32, i32], i64),
    "hvit_mhsa_keep_bits_used": ([i32, i32, i32], i32),
    "hvit_mhsa_fwd_kb": ([i32, vp, i32, i32, i32, i32, f32, P(Dropout), vp, vp, vp, vp], i32),
    "hvit_mhsa_bwd_kb": ([i32, vp, vp, vp, vp, i32, i32, i32, i32, f32, P(Dropout), vp, vp, vp, vp], i32),
    "hvit_mhsa_bwd_db": ([i32, vp, vp, vp, vp, i32, i32, i32, i32, f32, P(Dropout), vp, vp, vp, vp, vp], i32),
    "hvit_layernorm_fwd": ([vp, vp, vp, i32, i32, f32, vp, i32, vp, vp, vp], i32),
    "hvit_layernorm_bwd_ws_elems": ([i32, i32], i64),
    "hvit_layernorm_bwd_drop_ws_elems": ([i32, i32], i64),
    "hvit_layernorm_bwd_drop": ([vp, i32, vp, vp, vp, vp, i32, i32, vp, vp, vp, P(Dropout), vp, i32, vp, i32, vp,
                                 i64, i32, vp], i32),
    "hvit_layernorm_bwd": ([vp, i32, vp, vp, vp, vp, i32, i32, vp, vp, vp, vp, vp, i64, i32, vp], i32),
    "hvit_bn_finalize": ([vp, i32, i32, i64, i32, vp, vp, vp, vp, vp, f32, f32, vp], i32),
    "hvit_bn_eval_prep": ([vp, vp, i32, f32, vp, vp, vp], i32),
    "hvit_bn_act_fwd": ([i32, vp, i32, i32, i32, i32, vp, vp, vp, vp, P(Dropout), i32, vp, i32, vp], i32),
    "hvit_bn_act_bwd": ([i32, vp, i32, i32, i32, i32, vp, vp, vp, vp, P(Dropout), i32, vp, i32, i32, vp,
                         i32, vp, i32, vp], i32),
    "hvit_bn_act_bwd_sums_elems": ([i32], i64),
    "hvit_c1block_stats": ([i32, P(ConvGeom), vp, vp, vp], i32),
    "hvit_c1block_fwd": ([i32, P(ConvGeom), vp, vp, vp, vp, vp, P(Dropout), i32, vp, i32, vp], i32),
    "hvit_c1block_bwd_ws": ([P(ConvGeom), i32], i64),
    "hvit_c1block_bwd": ([i32, P(ConvGeom), vp, vp, vp, vp, vp, P(Dropout), i32, vp, i32, i32, vp, i32, vp, vp,
                          i64, vp], i32),
    "hvit_bilinear_fwd":([vp, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp], i32),
    "hvit_bilinear_bwd": ([vp, i32, i32, i32, i32, i32, i32, i32, vp, i32, i32, vp], i32),
    "hvit_upsample_split_bwd": ([vp, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp, i32, vp], i32),
    "hvit_cast": ([vp, i32, vp, i32, i64, vp], i32),
    "hvit_dropout_scale": ([vp, i32, i64, i32, P(Dropout), vp, i32, vp, i32, vp, vp, i64, vp], i32),
    "hvit_dropout_colsum_ws_elems": ([i32], i64),
    "hvit_tanh_bwd": ([vp, i32, vp, i64, vp, i32, vp], i32),
    "hvit_reduce_rows": ([vp, i32, i64, i64, i64, i32, vp, vp], i32),
    "hvit_sum_slabs": ([vp, i32, i64, vp, vp], i32),
    "hvit_droppath_scale": ([i32, P(Dropout), vp, vp], i32),
    "hvit_droppath_scales": ([i32, i32, P(Dropout), vp, vp], i32),
    "hvit_weight_prep": ([i32, P(WPrepItem), vp], i32),
    "hvit_conv_bn_tile_rows": ([P(ConvGeom)], i32),
    "hvit_loss_ws_elems": ([i32, i64], i64),
    "hvit_loss_fwd": ([vp, vp, i32, i64, P(LossCfg), vp, i64, vp, vp, vp], i32),
    "hvit_loss_bwd": ([vp, vp, i32, i64, P(LossCfg), vp, vp, vp, vp], i32),
    "hvit_clip_ws_elems": ([i32], i64),
    "hvit_clip_coef": ([i32, P(TensorRef), f32, vp, i64, vp, vp], i32),
    "hvit_scale_tensors": ([i32, P(TensorRef), vp, vp], i32),
    "hvit_adamw": ([i32, P(AdamWItem), P(AdamWHyper), vp, vp], i32),
    "hvit_adamw_dev": ([i32, P(AdamWItem), P(AdamWHyper), vp, vp, vp], i32),
    "hvit_rng_advance": ([vp, vp, vp], i32),
    "hvit_gemm_tune": ([i32, i32], i32),
    "hvit_probe_gemm_splitk": ([i32, i32, vp, vp, i32, i32, i32, i32, vp, i32, vp], i32),
    "hvit_step_bump": ([vp, i32, f32, vp], i32),
}

EXPORTED = sorted(k for k in _SIGS)

_lib = None
_lock = threading.Lock()


def lib():
    """Load libhvit.so once; raise loudly if it is absent."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"hvit: native library not found at {LIB_PATH}; run __graft_entry__.build() "
                        "(there is no CPU or PyTorch fallback for the HIP path)")
                h = C.CDLL(LIB_PATH)
                alt = "HVIT_LIB" in os.environ  # an older in-tree build for A/B: tolerate missing entry points
                for name, (args, res) in _SIGS.items():
                    if alt and not hasattr(h, name):
                        continue
                    fn = getattr(h, name)
                    fn.argtypes = args
                    fn.restype = res
                _lib = h
    return _lib


# Measurement hook (functional.py installs it): times a C-ABI call that no
# explicit op class covers, under the class "abi:<entry point>"
TIMER = None


def call(name, *args):
    if TIMER is not None:
        return TIMER(name, lambda: _call(name, *args))
    return _call(name, *args)


def _call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().hvit_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (code {rc}): {msg}")
    return rc


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(dev=None):
    """The current HIP stream of ``dev`` (default: the current device) as a raw
    pointer.  Straight from the C++ stream registry when torch exposes it: a
    ``torch.cuda.current_stream()`` object per launch is a measurable share of
    the per-step host enqueue time."""
    if _raw_stream is not None:
        if dev is None:
            idx = torch.cuda.current_device()
        elif isinstance(dev, torch.device):
            idx = dev.index if dev.index is not None else torch.cuda.current_device()
        else:
            idx = int(dev)
        return _raw_stream(idx)
    return torch.cuda.current_stream(dev).cuda_stream


def dt_of(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"hvit: unsupported dtype {t.dtype}")


def torch_dtype(dt: int):
    return torch.float32 if dt == F32 else torch.bfloat16


def ptr(t):
    return None if t is None else t.data_ptr()


def dropout(p=0.0, seed=0, site=0, seed_t=None) -> Dropout:
    """A dropout site.  ``seed_t`` (optional int64 device tensor of one word,
    a forward's seed written by hvit_rng_advance): the kernels use
    ``seed ^ seed_t[0]``; the struct keeps a reference so the word outlives it."""
    d = Dropout(float(p), int(seed) & 0xFFFFFFFFFFFFFFFF, int(site) & 0xFFFFFFFF,
                None if seed_t is None else seed_t.data_ptr())
    d.keep = seed_t
    return d
