"""CPU fp32 oracle for the HybridViT forward/backward hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this file;
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may use it, and there only as the checker / the timed CPU baseline.

This is a functional restatement of the reference model (aten ops on the CPU in
fp32, the same op sequence as the reference) written against a flat state dict
whose keys are the reference's 122 ``state_dict`` keys.  Every function cites the
reference lines it restates (paths relative to the reference repository root).

Parity pinning: the reference ships no tests or fixtures for this path, so the
oracle is pinned by golden vectors produced by importing the reference's own
``models`` package in the build container (``tools/gen_golden.py`` ->
``tests/golden/*.npz``); ``tests/test_oracle_golden.py`` checks this file against
them.  The backward is torch autograd over this restatement, exactly as the
reference's backward is autograd over its forward.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F


@dataclass
class HViTConfig:
    """Constructor arguments of ``HybridViT`` (models/hybrid_vit.py:36-67)."""

    input_channels: int = 1
    output_channels: int = 1
    encoder_channels: List[int] = field(default_factory=lambda: [64, 128, 256])
    encoder_kernel_sizes: List[int] = field(default_factory=lambda: [3, 3, 3])
    encoder_pool_sizes: List[int] = field(default_factory=lambda: [2, 2, 1])
    embed_dim: int = 512
    num_heads: int = 8
    num_layers: int = 6
    mlp_ratio: float = 4.0
    patch_size: int = 4
    decoder_channels: List[int] = field(default_factory=lambda: [256, 128, 64, 1])
    decoder_kernel_sizes: List[int] = field(default_factory=lambda: [3, 3, 3, 3])
    decoder_upsample_factors: List[int] = field(default_factory=lambda: [1, 2, 2, 1])
    dropout: float = 0.1
    attn_dropout: float = 0.1
    drop_path_rate: float = 0.1
    use_skip_connections: bool = True
    use_cls_token: bool = False

    def as_kwargs(self) -> dict:
        return dict(self.__dict__)


TINY = dict(encoder_channels=[8, 16, 32], embed_dim=64, num_heads=4, num_layers=2,
            decoder_channels=[32, 16, 8, 1])


def decoder_prefix(cfg: HViTConfig, i: int) -> Tuple[str, str]:
    """Sequential indices of the conv / BN inside TransposeConvBlock i.

    components.py:144-162: an ``nn.Upsample`` occupies index 0 when the block
    upsamples, shifting the conv to 1 and the BN to 2.
    """
    up = cfg.decoder_upsample_factors[i] > 1
    c = 1 if up else 0
    return f"decoder.{i}.block.{c}", f"decoder.{i}.block.{c + 1}"


def state_dict_shapes(cfg: HViTConfig) -> Dict[str, Tuple[int, ...]]:
    """The reference's state_dict keys and shapes in registration order
    (hybrid_vit.py:102-170, components.py, attention.py)."""
    s: Dict[str, Tuple[int, ...]] = {}
    if cfg.use_cls_token:  # a parameter of HybridViT itself: first in state_dict order
        s["cls_token"] = (1, 1, cfg.embed_dim)
    cin = cfg.input_channels
    for i, (co, k) in enumerate(zip(cfg.encoder_channels, cfg.encoder_kernel_sizes)):
        p = f"encoder.{i}.block"
        s[f"{p}.0.weight"] = (co, cin, k, k)
        for n in ("weight", "bias", "running_mean", "running_var"):
            s[f"{p}.1.{n}"] = (co,)
        s[f"{p}.1.num_batches_tracked"] = ()
        cin = co
    D, P = cfg.embed_dim, cfg.patch_size
    s["patch_embed.projection.weight"] = (D, cin, P, P)
    s["patch_embed.projection.bias"] = (D,)
    s["pos_encoding.pos_embed"] = (1, 10000, D)
    hid = int(D * cfg.mlp_ratio)
    for l in range(cfg.num_layers):
        p = f"transformer.blocks.{l}"
        for n in ("norm1", "norm2"):
            s[f"{p}.{n}.weight"] = (D,)
            s[f"{p}.{n}.bias"] = (D,)
        s[f"{p}.attn.qkv.weight"] = (3 * D, D)
        s[f"{p}.attn.qkv.bias"] = (3 * D,)
        s[f"{p}.attn.proj.weight"] = (D, D)
        s[f"{p}.attn.proj.bias"] = (D,)
        s[f"{p}.mlp.net.0.weight"] = (hid, D)
        s[f"{p}.mlp.net.0.bias"] = (hid,)
        s[f"{p}.mlp.net.3.weight"] = (D, hid)
        s[f"{p}.mlp.net.3.bias"] = (D,)
    s["transformer.norm.weight"] = (D,)
    s["transformer.norm.bias"] = (D,)
    enc_out = cfg.encoder_channels[-1]
    s["to_feature_map.weight"] = (enc_out, D)
    s["to_feature_map.bias"] = (enc_out,)
    dch = cfg.decoder_channels
    nd = len(dch)
    for i, (co, k) in enumerate(zip(dch, cfg.decoder_kernel_sizes)):
        in_ch = dch[0] if i == 0 else dch[i - 1]
        if cfg.use_skip_connections and i < nd - 1:
            in_ch += co
        conv, bn = decoder_prefix(cfg, i)
        s[f"{conv}.weight"] = (co, in_ch, k, k)
        if i < nd - 1:
            for n in ("weight", "bias", "running_mean", "running_var"):
                s[f"{bn}.{n}"] = (co,)
            s[f"{bn}.num_batches_tracked"] = ()
    if cfg.use_skip_connections:
        for i, (ec, dc) in enumerate(zip(cfg.encoder_channels[::-1], dch[:-1])):
            s[f"skip_projections.{i}.weight"] = (dc, ec, 1, 1)
            s[f"skip_projections.{i}.bias"] = (dc,)
    return s


# --------------------------------------------------------------------------- #
# forward restatement
# --------------------------------------------------------------------------- #

def _dropout(x, p, training, gen=None):
    # nn.Dropout (attention.py:61-62, components.py:226-228,340)
    return F.dropout(x, p, training) if p > 0 else x


def conv_block(sd, pfx, x, pool, p, training, momentum=0.1):
    """ConvBlock.forward (components.py:15-99): Conv(no bias) -> BN -> ReLU ->
    Dropout2d -> MaxPool."""
    w = sd[f"{pfx}.0.weight"]
    x = F.conv2d(x, w, None, 1, w.shape[-1] // 2)
    x = F.batch_norm(x, sd[f"{pfx}.1.running_mean"], sd[f"{pfx}.1.running_var"],
                     sd[f"{pfx}.1.weight"], sd[f"{pfx}.1.bias"], training, momentum, 1e-5)
    if training:
        sd[f"{pfx}.1.num_batches_tracked"] += 1
    x = F.relu(x)
    if p > 0:
        x = F.dropout2d(x, p, training)
    if pool is not None and pool > 1:
        x = F.max_pool2d(x, pool)
    return x


def tconv_block(sd, cfg, i, x, p, training, final):
    """TransposeConvBlock.forward (components.py:102-192): [nearest Up] -> Conv
    (no bias) -> BN -> ReLU -> Dropout2d ; final: Conv -> Tanh."""
    conv, bn = decoder_prefix(cfg, i)
    up = cfg.decoder_upsample_factors[i]
    if up > 1:
        x = F.interpolate(x, scale_factor=up, mode="nearest")
    w = sd[f"{conv}.weight"]
    x = F.conv2d(x, w, None, 1, w.shape[-1] // 2)
    if final:
        return torch.tanh(x)
    x = F.batch_norm(x, sd[f"{bn}.running_mean"], sd[f"{bn}.running_var"],
                     sd[f"{bn}.weight"], sd[f"{bn}.bias"], training, 0.1, 1e-5)
    if training:
        sd[f"{bn}.num_batches_tracked"] += 1
    x = F.relu(x)
    if p > 0:
        x = F.dropout2d(x, p, training)
    return x


def mhsa(sd, pfx, x, H, p_attn, p, training, want_attn=False):
    """MultiHeadSelfAttention.forward (attention.py:65-115)."""
    B, N, C = x.shape
    hd = C // H
    qkv = F.linear(x, sd[f"{pfx}.qkv.weight"], sd[f"{pfx}.qkv.bias"])
    qkv = qkv.reshape(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    attn = (q @ k.transpose(-2, -1)) * (hd ** -0.5)
    attn = attn.softmax(dim=-1)
    attn = _dropout(attn, p_attn, training)
    o = (attn @ v).transpose(1, 2).reshape(B, N, C)
    o = F.linear(o, sd[f"{pfx}.proj.weight"], sd[f"{pfx}.proj.bias"])
    o = _dropout(o, p, training)
    return (o, attn) if want_attn else (o, None)


def drop_path(x, prob, training):
    """DropPath.forward (components.py:407-427)."""
    if prob == 0.0 or not training:
        return x
    keep = 1 - prob
    r = keep + torch.rand((x.shape[0],) + (1,) * (x.ndim - 1), dtype=x.dtype)
    return x.div(keep) * r.floor_()


def vit_block(sd, pfx, x, cfg, dpr, training, want_attn=False):
    """TransformerEncoderBlock.forward (attention.py:176-213), pre-norm."""
    D = cfg.embed_dim
    h = F.layer_norm(x, (D,), sd[f"{pfx}.norm1.weight"], sd[f"{pfx}.norm1.bias"], 1e-5)
    a, attn = mhsa(sd, f"{pfx}.attn", h, cfg.num_heads, cfg.attn_dropout, cfg.dropout,
                   training, want_attn)
    x = x + drop_path(a, dpr, training)
    h = F.layer_norm(x, (D,), sd[f"{pfx}.norm2.weight"], sd[f"{pfx}.norm2.bias"], 1e-5)
    # FeedForward (components.py:223-241)
    h = F.linear(h, sd[f"{pfx}.mlp.net.0.weight"], sd[f"{pfx}.mlp.net.0.bias"])
    h = F.gelu(h)
    h = _dropout(h, cfg.dropout, training)
    h = F.linear(h, sd[f"{pfx}.mlp.net.3.weight"], sd[f"{pfx}.mlp.net.3.bias"])
    h = _dropout(h, cfg.dropout, training)
    x = x + drop_path(h, dpr, training)
    return x, attn


def forward(sd: Dict[str, torch.Tensor], x: torch.Tensor, cfg: HViTConfig,
            training: bool = False, return_attentions: bool = False,
            capture: Optional[dict] = None):
    """HybridViT.forward (hybrid_vit.py:396-469).

    ``capture`` (optional dict) receives named intermediates: ``enc{i}``,
    ``tokens`` (after patch embed), ``vit_out`` (after final LN), ``feat``
    (to_feature_map output as NCHW), ``pre_tanh`` and ``dec{i}``.
    """
    cap = capture if capture is not None else {}
    in_hw = x.shape[2:]
    # forward_encoder (hybrid_vit.py:286-307)
    skips = []
    for i, pool in enumerate(cfg.encoder_pool_sizes):
        x = conv_block(sd, f"encoder.{i}.block", x, pool if pool > 1 else None,
                       cfg.dropout, training)
        skips.append(x)
        cap[f"enc{i}"] = x
    # PatchEmbedding (components.py:282-307)
    P = cfg.patch_size
    t = F.conv2d(x, sd["patch_embed.projection.weight"], sd["patch_embed.projection.bias"],
                 P)
    B, D, Hp, Wp = t.shape
    t = t.flatten(2).transpose(1, 2)
    cap["tokens"] = t
    # forward_transformer (hybrid_vit.py:309-350) / return_attentions branch :422-453
    if cfg.use_cls_token:
        t = torch.cat([sd["cls_token"].expand(B, -1, -1), t], 1)
    N = t.shape[1]
    t = t + sd["pos_encoding.pos_embed"][:, :N, :]           # components.py:384
    t = _dropout(t, cfg.dropout, training)
    dpr = [v.item() for v in torch.linspace(0, cfg.drop_path_rate, cfg.num_layers)]
    attns = []
    for l in range(cfg.num_layers):
        t, a = vit_block(sd, f"transformer.blocks.{l}", t, cfg, dpr[l], training,
                         return_attentions)
        attns.append(a)
    t = F.layer_norm(t, (D,), sd["transformer.norm.weight"], sd["transformer.norm.bias"],
                     1e-5)
    cap["vit_out"] = t           # VisionTransformer output (CLS row included, as the reference module returns)
    if cfg.use_cls_token:
        t = t[:, 1:, :]          # hybrid_vit.py:337-338
    f = F.linear(t, sd["to_feature_map.weight"], sd["to_feature_map.bias"])
    C = f.shape[-1]
    x = f.transpose(1, 2).reshape(B, C, Hp, Wp)
    cap["feat"] = x
    # forward_decoder (hybrid_vit.py:352-394)
    skips = skips[::-1]
    nd = len(cfg.decoder_channels)
    for i in range(nd):
        if cfg.use_skip_connections and i < nd - 1 and i < len(skips):
            s = F.conv2d(skips[i], sd[f"skip_projections.{i}.weight"],
                         sd[f"skip_projections.{i}.bias"])
            if s.shape[2:] != x.shape[2:]:
                s = F.interpolate(s, size=x.shape[2:], mode="bilinear", align_corners=False)
            x = torch.cat([x, s], 1)
        final = i == nd - 1
        if final:
            conv, _ = decoder_prefix(cfg, i)
            up = cfg.decoder_upsample_factors[i]
            if up > 1:
                x = F.interpolate(x, scale_factor=up, mode="nearest")
            w = sd[f"{conv}.weight"]
            z = F.conv2d(x, w, None, 1, w.shape[-1] // 2)
            cap["pre_tanh"] = z
            x = torch.tanh(z)
        else:
            x = tconv_block(sd, cfg, i, x, cfg.dropout, training, False)
        cap[f"dec{i}"] = x
    # final resize (hybrid_vit.py:459-465)
    if tuple(x.shape[2:]) != tuple(in_hw):
        x = F.interpolate(x, size=tuple(in_hw), mode="bilinear", align_corners=False)
    if return_attentions:
        return x, attns
    return x


def combined_loss(pred, target, l1_weight=1.0, stoi_weight=0.1, mse_weight=0.0, perceptual_weight=0.0,
                  use_log_compression=False, return_components=False):
    """CombinedLoss.forward (training/losses.py:330-387); defaults are those of
    create_loss_function (:390-408).  l1·L1 + mse·MSE on log(x + 1e-8) when
    use_log_compression (:319-321, :344-346), + stoi·mean(1 - cos(flat(p),
    flat(t))) (STOILoss :109-141, on the uncompressed inputs) + perceptual·L1
    (PerceptualLoss :270-283, placeholder L1 on the uncompressed inputs)."""
    pi, ti = (torch.log(pred + 1e-8), torch.log(target + 1e-8)) if use_log_compression else (pred, target)
    total = 0.0
    comps = {}
    if l1_weight > 0:
        l1 = (pi - ti).abs().mean()
        comps["l1"] = l1
        total = total + l1_weight * l1
    if mse_weight > 0:
        mse = ((pi - ti) ** 2).mean()
        comps["mse"] = mse
        total = total + mse_weight * mse
    if stoi_weight > 0:
        pn = F.normalize(pred.flatten(1), dim=1)
        tn = F.normalize(target.flatten(1), dim=1)
        stoi = (1.0 - (pn * tn).sum(1)).mean()
        comps["stoi"] = stoi
        total = total + stoi_weight * stoi
    if perceptual_weight > 0:
        perc = (pred - target).abs().mean()
        comps["perceptual"] = perc
        total = total + perceptual_weight * perc
    return (total, comps) if return_components else total


def is_buffer(key: str) -> bool:
    return "running_" in key or key.endswith("num_batches_tracked")


def make_state(shapes: Dict[str, Tuple[int, ...]], values: Dict[str, "np.ndarray"], requires_grad=False):
    """Tensors for ``forward`` (float32; num_batches_tracked as int64).  With
    ``requires_grad`` the parameters (not the BN buffers) track gradients."""
    sd = {}
    for k, shp in shapes.items():
        if k.endswith("num_batches_tracked"):
            sd[k] = torch.zeros((), dtype=torch.int64)
        else:
            sd[k] = torch.as_tensor(values[k], dtype=torch.float32).reshape(shp).clone()
            if requires_grad and not is_buffer(k):
                sd[k].requires_grad_(True)
    return sd
