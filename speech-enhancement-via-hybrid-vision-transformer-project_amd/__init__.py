"""MI355X-native HybridViT hot path (gfx950 HIP kernels behind the reference's
nn.Module API).  Import name when loaded by the repository helpers: ``hvit_amd``.

Public surface (mirrors the reference's ``models`` package, models/__init__.py,
plus the factory it forgot to export):
    HybridViT, create_hybrid_vit, ConvBlock, TransposeConvBlock, FeedForward,
    PatchEmbedding, PositionalEncoding, MultiHeadSelfAttention,
    TransformerEncoderBlock, VisionTransformer, CombinedLoss, create_loss_function,
    FusedAdamW / clip_grad_norm_ / create_optimizer (training/optimizer.py, trainer.py:170-174),
    GraphedTrainStep (the train step replayed from a hipGraph per input shape, trainer.py:142-183)
"""

from .hybrid_vit import (  # noqa: F401
    ConvBlock,
    DropPath,
    FeedForward,
    HybridViT,
    MultiHeadSelfAttention,
    PatchEmbedding,
    PositionalEncoding,
    TransformerEncoderBlock,
    TransposeConvBlock,
    VisionTransformer,
    create_hybrid_vit,
)
from .losses import CombinedLoss, create_loss_function  # noqa: F401
from .optim import FusedAdamW, clip_grad_norm_, create_optimizer  # noqa: F401
from .train_step import GraphedTrainStep  # noqa: F401
from .config import load_all_configs, load_config, merge_configs  # noqa: F401
from . import _lib  # noqa: F401

__all__ = [
    "HybridViT", "create_hybrid_vit", "ConvBlock", "TransposeConvBlock", "FeedForward", "PatchEmbedding",
    "PositionalEncoding", "MultiHeadSelfAttention", "TransformerEncoderBlock", "VisionTransformer",
    "CombinedLoss", "create_loss_function", "FusedAdamW", "clip_grad_norm_", "create_optimizer", "GraphedTrainStep",
    "load_all_configs", "load_config", "merge_configs",
]
