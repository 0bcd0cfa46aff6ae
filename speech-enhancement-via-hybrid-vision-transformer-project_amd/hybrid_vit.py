"""Drop-in ``HybridViT`` (reference: models/hybrid_vit.py, models/attention.py,
models/components.py) whose forward/backward run on libhvit.so (gfx950).

The constructor signature and defaults, the submodule tree, parameter names,
the 122 ``state_dict`` keys and shapes, the weight initialisation,
``forward(x, return_attentions=False)``, ``forward_encoder`` /
``forward_transformer`` / ``forward_decoder``, ``count_parameters`` and
``create_hybrid_vit(config)`` all follow the reference, so reference
checkpoints load with ``strict=True`` and Trainer / AudioEnhancer callers work
unchanged.  The torch submodules (Conv2d, BatchNorm2d, LayerNorm, Linear) are
kept as parameter containers only: their ``forward`` is never called.

Precision: ``precision="fp32"`` runs the exact-f32 MFMA path (parity with the
reference within 1e-3 rel); ``"bf16"`` runs bf16 MFMA with f32 accumulation, f32
residual stream / statistics / weight gradients; ``"auto"`` (default) picks bf16
inside a CUDA autocast region (the reference's trainer.py:148 AMP context) and
fp32 otherwise.  ``attention_precision="fp8"`` (an extra keyword; the
reference's keywords and defaults are unchanged) runs the attention forward of
the bf16 path on e4m3 MFMAs (BASELINE config 5, csrc/attention_fp8.hip) with
the bf16 attention backward.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib as L
from . import functional as HF


# ------------------------------------------------------------ containers ----
class ConvBlock(nn.Module):
    """components.py:15-99 (Conv no-bias, BN, ReLU, Dropout2d, MaxPool)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, pool_size=2,
                 activation="relu", use_batchnorm=True, dropout=0.0):
        super().__init__()
        if activation != "relu" or not use_batchnorm or stride != 1 or padding != kernel_size // 2:
            raise NotImplementedError("hvit ConvBlock: relu + batchnorm same-conv only (the HybridViT use)")
        if pool_size not in (None, 1, 2):
            raise NotImplementedError("hvit ConvBlock: pool_size must be 1 or 2")
        layers = [nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=False),
                  nn.BatchNorm2d(out_channels), nn.ReLU(inplace=True)]
        if dropout > 0:
            layers.append(nn.Dropout2d(dropout))
        if pool_size is not None and pool_size > 1:
            layers.append(nn.MaxPool2d(kernel_size=pool_size))
        self.block = nn.Sequential(*layers)
        self.pool = pool_size if (pool_size is not None and pool_size > 1) else 1
        self.p = dropout

    @property
    def conv(self):
        return self.block[0]

    @property
    def bn(self):
        return self.block[1]


class TransposeConvBlock(nn.Module):
    """components.py:102-192 ([nearest Up], Conv no-bias, BN / Tanh, ReLU, Dropout2d)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, output_padding=0,
                 upsample_factor=2, activation="relu", use_batchnorm=True, dropout=0.0, final_layer=False):
        super().__init__()
        if activation != "relu" or not use_batchnorm or stride != 1 or padding != kernel_size // 2:
            raise NotImplementedError("hvit TransposeConvBlock: relu + batchnorm same-conv only")
        layers = []
        self.up = upsample_factor if (upsample_factor is not None and upsample_factor > 1) else 1
        if self.up > 1:
            layers.append(nn.Upsample(scale_factor=upsample_factor, mode="nearest"))
        layers.append(nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=False))
        if not final_layer:
            layers.append(nn.BatchNorm2d(out_channels))
        layers.append(nn.Tanh() if final_layer else nn.ReLU(inplace=True))
        if dropout > 0 and not final_layer:
            layers.append(nn.Dropout2d(dropout))
        self.block = nn.Sequential(*layers)
        self.final = final_layer
        self.p = dropout if not final_layer else 0.0

    @property
    def conv(self):
        return self.block[1 if self.up > 1 else 0]

    @property
    def bn(self):
        return self.block[2 if self.up > 1 else 1]


class PatchEmbedding(nn.Module):
    """components.py:244-307."""

    def __init__(self, in_channels, embed_dim, patch_size=4, flatten=True):
        super().__init__()
        self.patch_size = patch_size
        self.flatten = flatten
        self.projection = nn.Conv2d(in_channels, embed_dim, kernel_size=patch_size, stride=patch_size)


class PositionalEncoding(nn.Module):
    """components.py:310-386 (learnable table, the HybridViT configuration)."""

    def __init__(self, embed_dim, max_len=5000, learnable=True, dropout=0.1):
        super().__init__()
        if not learnable:
            raise NotImplementedError("hvit: HybridViT uses the learnable positional table")
        self.embed_dim = embed_dim
        self.learnable = learnable
        self.dropout = nn.Dropout(dropout)
        self.pos_embed = nn.Parameter(torch.zeros(1, max_len, embed_dim))
        nn.init.trunc_normal_(self.pos_embed, std=0.02)


class DropPath(nn.Module):
    """components.py:389-427 (per-sample stochastic depth)."""

    def __init__(self, drop_prob=0.0):
        super().__init__()
        self.drop_prob = drop_prob


class FeedForward(nn.Module):
    """components.py:195-241."""

    def __init__(self, dim, hidden_dim=None, dropout=0.0):
        super().__init__()
        hidden_dim = hidden_dim or 4 * dim
        self.net = nn.Sequential(nn.Linear(dim, hidden_dim), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hidden_dim, dim), nn.Dropout(dropout))


class MultiHeadSelfAttention(nn.Module):
    """attention.py:17-115."""

    def __init__(self, embed_dim, num_heads=8, qkv_bias=True, attn_dropout=0.0, proj_dropout=0.0):
        super().__init__()
        assert embed_dim % num_heads == 0, \
            f"embed_dim ({embed_dim}) must be divisible by num_heads ({num_heads})"
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        if self.head_dim not in (16, 32, 64):
            raise NotImplementedError(f"hvit: head_dim {self.head_dim} unsupported (16, 32, 64)")
        self.scale = self.head_dim ** -0.5
        if not qkv_bias:
            raise NotImplementedError("hvit: qkv_bias=False unsupported")
        self.qkv = nn.Linear(embed_dim, embed_dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(embed_dim, embed_dim)
        self.attn_dropout = nn.Dropout(attn_dropout)
        self.proj_dropout = nn.Dropout(proj_dropout)


class TransformerEncoderBlock(nn.Module):
    """attention.py:118-213 (pre-norm)."""

    def __init__(self, embed_dim, num_heads=8, mlp_ratio=4.0, qkv_bias=True, dropout=0.0, attn_dropout=0.0,
                 drop_path=0.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(embed_dim)
        self.norm2 = nn.LayerNorm(embed_dim)
        self.attn = MultiHeadSelfAttention(embed_dim, num_heads, qkv_bias, attn_dropout, dropout)
        self.mlp = FeedForward(embed_dim, int(embed_dim * mlp_ratio), dropout)
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        self.dpr = drop_path
        self.p = dropout
        self.p_attn = attn_dropout


class VisionTransformer(nn.Module):
    """attention.py:216-304."""

    def __init__(self, embed_dim, num_layers=6, num_heads=8, mlp_ratio=4.0, qkv_bias=True, dropout=0.0,
                 attn_dropout=0.0, drop_path_rate=0.0):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_layers = num_layers
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, num_layers)]
        self.blocks = nn.ModuleList([
            TransformerEncoderBlock(embed_dim, num_heads, mlp_ratio, qkv_bias, dropout, attn_dropout, dpr[i])
            for i in range(num_layers)])
        self.norm = nn.LayerNorm(embed_dim)


def _on_input_device(fn):
    """Run a forward entry point under a device guard for its input tensor."""
    import functools

    @functools.wraps(fn)
    def run(self, x, *a, **k):
        if isinstance(x, torch.Tensor) and x.is_cuda:
            with torch.cuda.device(x.device):
                return fn(self, x, *a, **k)
        return fn(self, x, *a, **k)

    return run


# ------------------------------------------------------------------ model ---
class HybridViT(nn.Module):
    """HybridViT (models/hybrid_vit.py:21-489) on the gfx950 HIP path."""

    def __init__(
        self,
        input_channels: int = 1,
        output_channels: int = 1,
        encoder_channels: List[int] = [64, 128, 256],
        encoder_kernel_sizes: List[int] = [3, 3, 3],
        encoder_pool_sizes: List[int] = [2, 2, 1],
        embed_dim: int = 512,
        num_heads: int = 8,
        num_layers: int = 6,
        mlp_ratio: float = 4.0,
        patch_size: int = 4,
        decoder_channels: List[int] = [256, 128, 64, 1],
        decoder_kernel_sizes: List[int] = [3, 3, 3, 3],
        decoder_upsample_factors: List[int] = [1, 2, 2, 1],
        dropout: float = 0.1,
        attn_dropout: float = 0.1,
        drop_path_rate: float = 0.1,
        use_skip_connections: bool = True,
        use_cls_token: bool = False,
        precision: str = "auto",
        attention_precision: Optional[str] = None,
    ):
        super().__init__()
        self.input_channels = input_channels
        self.output_channels = output_channels
        self.embed_dim = embed_dim
        self.patch_size = patch_size
        self.use_skip_connections = use_skip_connections
        self.use_cls_token = use_cls_token
        self.num_heads = num_heads
        self.dropout_p = dropout
        self.precision = precision
        if attention_precision not in (None, "fp8"):
            raise ValueError(f"hvit: attention_precision must be None or 'fp8', got {attention_precision!r}")
        # "fp8": e4m3 QK^T / PV MFMAs in the attention forward of the bf16 path
        # (BASELINE config 5); the attention backward stays bf16
        if attention_precision == "fp8" and precision in ("fp32", "float32"):
            raise ValueError("hvit: attention_precision='fp8' runs inside the bf16 path; precision='fp32' "
                             "cannot use it (use precision='bf16' or 'auto' under autocast)")
        self.attention_precision = attention_precision
        self._fp8_warned = False
        self.last_num_tokens = 0  # patch tokens N of the latest forward (dp.GradAllReducer checks it)

        self.encoder = nn.ModuleList()
        in_ch = input_channels
        for out_ch, k, pool in zip(encoder_channels, encoder_kernel_sizes, encoder_pool_sizes):
            self.encoder.append(ConvBlock(in_ch, out_ch, k, padding=k // 2, pool_size=pool if pool > 1 else None,
                                          dropout=dropout))
            in_ch = out_ch
        enc_out = encoder_channels[-1]
        self.patch_embed = PatchEmbedding(enc_out, embed_dim, patch_size, flatten=True)
        if use_cls_token:  # hybrid_vit.py:118-123 (never set by create_hybrid_vit; off the hot path)
            self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
            nn.init.trunc_normal_(self.cls_token, std=0.02)
        else:
            self.cls_token = None
        self.pos_encoding = PositionalEncoding(embed_dim, max_len=10000, learnable=True, dropout=dropout)
        self.transformer = VisionTransformer(embed_dim, num_layers, num_heads, mlp_ratio, True, dropout,
                                             attn_dropout, drop_path_rate)
        self.to_feature_map = nn.Linear(embed_dim, enc_out)
        self.decoder = nn.ModuleList()
        nd = len(decoder_channels)
        for i, (out_ch, k, up) in enumerate(zip(decoder_channels, decoder_kernel_sizes,
                                                decoder_upsample_factors)):
            in_c = decoder_channels[0] if i == 0 else decoder_channels[i - 1]
            if use_skip_connections and i < nd - 1:
                in_c = in_c + out_ch
            final = i == nd - 1
            self.decoder.append(TransposeConvBlock(in_c, out_ch, k, padding=k // 2,
                                                   upsample_factor=up if up > 1 else None,
                                                   dropout=dropout if not final else 0.0, final_layer=final))
        if use_skip_connections:
            self.skip_projections = nn.ModuleList([
                nn.Conv2d(ec, dc, kernel_size=1) for ec, dc in zip(encoder_channels[::-1], decoder_channels[:-1])])
        else:
            self.skip_projections = None
        self.apply(self._init_weights)

    @staticmethod
    def _init_weights(m):
        """hybrid_vit.py:265-284."""
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, (nn.BatchNorm2d, nn.LayerNorm)):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)

    # -------------------------------------------------------------- helpers --
    def _dt(self) -> int:
        p = self.precision
        if p == "auto":
            return L.BF16 if torch.is_autocast_enabled("cuda") else L.F32
        if p in ("bf16", "bfloat16"):
            return L.BF16
        if p in ("fp32", "float32"):
            return L.F32
        raise ValueError(f"hvit: unknown precision {p!r}")

    def _check_device(self, x):
        if not x.is_cuda:
            raise RuntimeError("hvit: the HIP path needs GPU tensors (call .to('cuda')); there is no CPU path")
        lib = L.lib()  # noqa: F841  (fails loudly when libhvit.so is missing)
        # the (name, parameter) list is cached (walking the module tree every
        # forward was ~0.4 ms of host time per step); _apply (.to / .cuda / ...)
        # drops it
        named = self.__dict__.get("_hvit_named_params")
        if named is None:
            named = list(self.named_parameters())
            self.__dict__["_hvit_named_params"] = named
        dev = x.device
        for n, t in named:
            if t.device != dev:
                raise RuntimeError(f"hvit: input on {x.device} but parameter {n} on {t.device}")

    def _apply(self, fn, *args, **kwargs):
        self.__dict__.pop("_hvit_named_params", None)
        return super()._apply(fn, *args, **kwargs)

    def _seed(self) -> Optional[torch.Tensor]:
        """This training forward's dropout seed, as a one-word device tensor
        (None in eval).  The seed stream lives on the device: a state
        {base, counter} that hvit_rng_advance steps once per training forward,
        writing the new seed to a fresh word that this forward's dropout sites
        (and their backward) read.  So a captured train step (hipGraph) draws new
        masks on every replay, and the masks of a replay sequence equal those of
        the same number of eager steps from the same state.  ``base`` is drawn
        from torch's host generator whenever that generator was re-seeded or
        used since the previous draw (checked on eager forwards only), so
        ``torch.manual_seed`` makes the dropout of the next forward
        reproducible as with the reference's torch dropout."""
        if not self.training:
            return None
        dev = torch.device("cuda", torch.cuda.current_device())
        st = self.__dict__.get("_rng_state")
        if st is None or st.device != dev:
            st = torch.zeros(2, dtype=torch.int64, device=dev)
            self.__dict__["_rng_state"] = st
            self.__dict__["_rng_host"] = None
        if not torch.cuda.is_current_stream_capturing():
            gen = torch.default_generator
            hs = self.__dict__.get("_rng_host")
            if hs is None or not torch.equal(gen.get_state(), hs):
                base = int(torch.randint(0, 2 ** 62, (1,)).item())
                st[0].fill_(base)  # fill kernels: no host-device synchronisation
                st[1].zero_()
                self.__dict__["_rng_host"] = gen.get_state()
        seed_t = torch.empty(1, dtype=torch.int64, device=dev)
        L.call("hvit_rng_advance", st.data_ptr(), seed_t.data_ptr(), L.stream_ptr())
        return seed_t

    def set_dropout_state(self, base: int, counter: int = 0) -> None:
        """Reset the device dropout seed stream (see _seed) to {base, counter}."""
        dev = torch.device("cuda", torch.cuda.current_device())
        st = torch.tensor([int(base) & 0x7FFFFFFFFFFFFFFF, int(counter)], dtype=torch.int64).to(dev)
        self.__dict__["_rng_state"] = st
        self.__dict__["_rng_host"] = torch.default_generator.get_state()

    def dropout_state(self) -> Optional[torch.Tensor]:
        """A copy of the device dropout seed state {base, counter} (None before
        the first training forward)."""
        st = self.__dict__.get("_rng_state")
        return None if st is None else st.clone()

    def train(self, mode: bool = True):
        """nn.Module.train / eval; also drops the prepared-weight cache (inference
        forwards reuse packed / BN-folded weights only within one eval period)."""
        HF.prep_cache_clear()
        return super().train(mode)

    def _prep_weights(self, dt: int, dev) -> None:
        """Cast / pack every weight this forward (and its backward) will use
        in one multi-tensor launch instead of one launch per weight."""
        grads = torch.is_grad_enabled()
        # inference (eval, no grad): the conv blocks' eval BatchNorm folded into their packed weights in the
        # same launch (kind 3; HF.ConvBNActFn takes it) -- a pooling block also keeps the plain packing, used
        # should the pooled fused form not apply to the input's shape
        fold = not grads and not self.training and HF.EVALFOLD

        def conv_items(blk, plain):
            bn = blk.bn
            w = blk.conv.weight
            out = [(w, 3, dt, (bn.weight, bn.bias, bn.running_mean, bn.running_var, float(bn.eps)))]
            return out + [(w, 1, dt)] if plain else out

        items = []
        for i, blk in enumerate(self.encoder):
            if fold and i > 0:
                items += conv_items(blk, blk.pool != 1)
            else:
                items.append((blk.conv.weight, 1, dt))
            if grads and i > 0:
                items.append((blk.conv.weight, 2, dt))
        items.append((self.patch_embed.projection.weight, 1, dt))
        for blk in self.transformer.blocks:
            items += [(blk.attn.qkv.weight, 0, dt), (blk.attn.proj.weight, 0, dt),
                      (blk.mlp.net[0].weight, 0, dt), (blk.mlp.net[3].weight, 0, dt)]
        items.append((self.to_feature_map.weight, 0, dt))
        if self.use_skip_connections:
            items += [(sp.weight, 0, dt) for sp in self.skip_projections]
        for blk in self.decoder:
            if fold and not blk.final:
                items += conv_items(blk, False)
            else:
                items.append((blk.conv.weight, 1, dt))
            if grads:
                items.append((blk.conv.weight, 2, dt))
        HF.prep_weights(items, dev, reuse=fold)

    @staticmethod
    def _nhwc(t: torch.Tensor) -> torch.Tensor:
        """NCHW logical tensor (possibly a channels-last view) -> NHWC contiguous."""
        return t.permute(0, 2, 3, 1).contiguous()

    @staticmethod
    def _nchw(t: torch.Tensor) -> torch.Tensor:
        """NHWC storage -> NCHW logical view (channels-last strides, no copy)."""
        return t.permute(0, 3, 1, 2)

    # ---------------------------------------------------------- stage runners --
    def _encoder(self, xh, dt, seed, sgs=None):
        """Encoder blocks; each output is a skip.  sgs (full forward only): one
        HF.SkipGrad per encoder output, through which the output's SkipFn hands
        its gradient to the output's other consumer (next block / patch embed)
        instead of an autograd add."""
        skips = []
        h = xh
        for i, blk in enumerate(self.encoder):
            bn = blk.bn
            sg = sgs[i - 1] if sgs is not None and i > 0 else None  # this block consumes output i - 1
            if HF.c1block_ok(h, None, blk.conv.weight, 1, blk.pool):
                h = HF.C1BlockFn.apply(h, blk.conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                       bn.num_batches_tracked, blk.pool, self.training,
                                       HF.Drop(blk.p, 0, 100 + i, seed), bn.momentum, bn.eps, dt)
            else:
                h = HF.ConvBNActFn.apply(h, None, blk.conv.weight, bn.weight, bn.bias, bn.running_mean,
                                         bn.running_var, bn.num_batches_tracked, 1, blk.pool, self.training,
                                         HF.Drop(blk.p, 0, 100 + i, seed), bn.momentum, bn.eps, dt, sg,
                                         not torch.is_grad_enabled())
            skips.append(h)
        return h, skips

    def _tokens(self, feat, dt, seed, sg=None):
        P = self.patch_size
        pe = self.patch_embed.projection
        hw = (feat.shape[1] // P, feat.shape[2] // P)
        if self.cls_token is None:  # hot path: pos-embed add and dropout fused into the GEMM epilogue
            t = HF.PatchEmbedFn.apply(feat, pe.weight, pe.bias, self.pos_encoding.pos_embed, P,
                                      HF.Drop(self.dropout_p, 0, 200, seed), self.training, dt, sg)
            self.last_num_tokens = t.shape[1]
            return t, hw
        t = HF.PatchEmbedFn.apply(feat, pe.weight, pe.bias, None, P, HF.Drop(), False, dt, sg)
        return self._pos_tokens(t, seed), hw

    def _pos_tokens(self, t, seed):
        """[CLS +] pos_embed[:, :N] + dropout on given tokens (hybrid_vit.py:323-333,
        components.py:371-386); same counter-hash mask (site 200) as the fused path."""
        if self.cls_token is not None:
            t = torch.cat([self.cls_token.expand(t.shape[0], -1, -1).float(), t.float()], 1)
        self.last_num_tokens = t.shape[1]
        return HF.PosDropFn.apply(t, self.pos_encoding.pos_embed, HF.Drop(self.dropout_p, 0, 200, seed), self.training)

    def _vit(self, t, dt, seed, want_attn=False):
        """Returns (tokens, attention maps, the last block's GradHandoff or None).
        Each block's fc2-branch dropout backward rides on the next block's LN1
        backward (HF.GradHandoff)."""
        attns = []
        ho = None
        if self.attention_precision == "fp8" and dt != L.BF16 and not self._fp8_warned:
            import warnings
            warnings.warn("hvit: attention_precision='fp8' is ignored: this forward runs the fp32 path "
                          "(precision='auto' outside an autocast region)")
            self._fp8_warned = True
        dps = [HF.Drop(0.0, (300 + 10 * l) << 20, 1, seed) for l in range(len(self.transformer.blocks))]
        if self.training:  # every block's DropPath multipliers from one launch
            HF.droppath_scales_all(t.shape[0], [(blk.dpr, d) for blk, d in zip(self.transformer.blocks, dps)],
                                   t.device)
        for l, blk in enumerate(self.transformer.blocks):
            a, m = blk.attn, blk.mlp.net
            base = 300 + 10 * l
            drops = (HF.Drop(blk.p_attn, 0, base, seed), HF.Drop(blk.p, 0, base + 1, seed),
                     HF.Drop(blk.p, 0, base + 2, seed), HF.Drop(blk.p, 0, base + 3, seed), dps[l])
            ho_in, ho = ho, (HF.GradHandoff() if HF.LNDROP and self.training else None)
            t, probs = HF.ViTBlockFn.apply(t, blk.norm1.weight, blk.norm1.bias, a.qkv.weight, a.qkv.bias,
                                           a.proj.weight, a.proj.bias, blk.norm2.weight, blk.norm2.bias,
                                           m[0].weight, m[0].bias, m[3].weight, m[3].bias, a.num_heads, drops,
                                           blk.dpr, self.training, dt, want_attn,
                                           self.attention_precision == "fp8" and dt == L.BF16, ho_in, ho,
                                           not torch.is_grad_enabled())
            attns.append(probs)
        return t, attns, ho

    def _head(self, t, hw, dt, ho=None):
        if self.cls_token is not None:
            t = t[:, 1:]  # hybrid_vit.py:337-338 (LayerNorm is per token, so dropping first is equivalent)
            ho = None  # the handoff's row -> sample map covers the cls row
        n = self.transformer.norm
        return HF.HeadFn.apply(t, n.weight, n.bias, self.to_feature_map.weight, self.to_feature_map.bias, hw, dt,
                               ho)

    def _decoder(self, x, skips, out_hw, dt, seed, sgs=None):
        skips = skips[::-1]
        sgs = sgs[::-1] if sgs is not None else [None] * len(skips)
        nd = len(self.decoder)
        for i, blk in enumerate(self.decoder):
            if blk.final:
                return HF.FinalFn.apply(x, blk.conv.weight, blk.up, out_hw, dt)
            s = None
            if self.use_skip_connections and i < nd - 1 and i < len(skips):
                sp = self.skip_projections[i]
                s = HF.SkipFn.apply(skips[i], sp.weight, sp.bias, x.shape[1], x.shape[2], dt, sgs[i])
            bn = blk.bn
            x = HF.ConvBNActFn.apply(x, s, blk.conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                     bn.num_batches_tracked, blk.up, 1, self.training,
                                     HF.Drop(blk.p, 0, 500 + i, seed), bn.momentum, bn.eps, dt, None,
                                     not torch.is_grad_enabled())
        raise RuntimeError("hvit: decoder has no final layer")

    # -------------------------------------------------------- reference API --
    @_on_input_device
    def forward_encoder(self, x: torch.Tensor) -> Tuple[torch.Tensor, List[torch.Tensor]]:
        """hybrid_vit.py:286-307.  Returns NCHW views (channels-last storage)."""
        self._check_device(x)
        dt = self._dt()
        h, skips = self._encoder(HF.CastFn.apply(self._nhwc(x), dt), dt, self._seed())
        HF.zflush(x.device)
        return self._nchw(h), [self._nchw(s) for s in skips]

    @_on_input_device
    def forward_transformer(self, x: torch.Tensor, spatial_shape: Tuple[int, int]) -> torch.Tensor:
        """hybrid_vit.py:309-350: patch tokens [B, N, D] (without pos-enc) -> [B, C, H, W]."""
        self._check_device(x)
        dt = self._dt()
        seed = self._seed()
        t = self._pos_tokens(x, seed)
        t, _, ho = self._vit(t, dt, seed)
        out = self._head(t, spatial_shape, dt, ho)
        HF.zflush(x.device)
        return self._nchw(out)

    @_on_input_device
    def forward_decoder(self, x: torch.Tensor, skip_features: List[torch.Tensor]) -> torch.Tensor:
        """hybrid_vit.py:352-394 (output before the final resize)."""
        self._check_device(x)
        dt = self._dt()
        xh = HF.CastFn.apply(self._nhwc(x), dt)
        skips = [HF.CastFn.apply(self._nhwc(s), dt) for s in skip_features]
        U = self.decoder[-1].up
        H = xh.shape[1]
        W = xh.shape[2]
        for blk in self.decoder[:-1]:
            H, W = H * blk.up, W * blk.up
        out = self._decoder(xh, skips, (H * U, W * U), dt, self._seed())
        HF.zflush(x.device)
        return self._nchw(out)

    def forward(self, x: torch.Tensor, return_attentions: bool = False):
        """hybrid_vit.py:396-469.  Kernels are launched on ``x``'s device (a
        device guard, so a model on cuda:1 works while cuda:0 is current; the
        autograd engine runs the backward on the same device)."""
        self._check_device(x)
        with torch.cuda.device(x.device):
            return self._forward(x, return_attentions)

    def _forward(self, x: torch.Tensor, return_attentions: bool):
        if x.dim() != 4:
            raise ValueError(f"hvit: expected [B, C, F, T], got {tuple(x.shape)}")
        dt = self._dt()
        seed = self._seed()
        F, T = x.shape[2], x.shape[3]
        self._prep_weights(dt, x.device)
        xh = HF.CastFn.apply(self._nhwc(x.float() if x.dtype != torch.float32 else x), dt)
        # skip gradients handed between an encoder output's two consumers (HF.SkipGrad)
        sgs = [HF.SkipGrad() for _ in self.encoder] if self.use_skip_connections and HF.SKIPGRAD else None
        feat, skips = self._encoder(xh, dt, seed, sgs)
        t, hw = self._tokens(feat, dt, seed, sgs[-1] if sgs else None)
        t, attns, ho = self._vit(t, dt, seed, return_attentions)
        f = self._head(t, hw, dt, ho)
        out = self._decoder(f, skips, (F, T), dt, seed, sgs)
        HF.zflush(x.device)
        out = self._nchw(out)
        if return_attentions:
            return out, attns
        return out

    def count_parameters(self) -> Dict[str, int]:
        """hybrid_vit.py:471-489."""
        return {
            "encoder": sum(p.numel() for p in self.encoder.parameters()),
            "transformer": sum(p.numel() for p in self.transformer.parameters()),
            "decoder": sum(p.numel() for p in self.decoder.parameters()),
            "total": sum(p.numel() for p in self.parameters()),
            "trainable": sum(p.numel() for p in self.parameters() if p.requires_grad),
        }


def create_hybrid_vit(config: Optional[Dict] = None, **overrides) -> HybridViT:
    """hybrid_vit.py:492-525 (same config keys and defaults)."""
    config = config or {}
    mc = config.get("model", {})
    enc, tr, dec = mc.get("encoder", {}), mc.get("transformer", {}), mc.get("decoder", {})
    kw = dict(
        input_channels=mc.get("input_channels", 1),
        output_channels=mc.get("output_channels", 1),
        encoder_channels=enc.get("channels", [64, 128, 256]),
        encoder_kernel_sizes=enc.get("kernel_sizes", [3, 3, 3]),
        encoder_pool_sizes=enc.get("pool_sizes", [2, 2, 1]),
        embed_dim=tr.get("embed_dim", 512),
        num_heads=tr.get("num_heads", 8),
        num_layers=tr.get("num_layers", 6),
        mlp_ratio=tr.get("mlp_ratio", 4),
        patch_size=tr.get("patch_size", 4),
        decoder_channels=dec.get("channels", [256, 128, 64, 1]),
        decoder_kernel_sizes=dec.get("kernel_sizes", [3, 3, 3, 3]),
        decoder_upsample_factors=dec.get("upsample_factors", [1, 2, 2, 1]),
        dropout=enc.get("dropout", 0.1),
        attn_dropout=tr.get("attention_dropout", 0.1),
        drop_path_rate=tr.get("drop_path_rate", 0.1),
        use_skip_connections=dec.get("use_skip_connections", True),
    )
    kw.update(overrides)
    return HybridViT(**kw)
