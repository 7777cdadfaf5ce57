"""Hot ops of the framework. GPU (bf16) tensors run hand-written gfx950 HIP
kernels from ``csrc/kernels``; CPU tensors run fp32 PyTorch references."""
from . import _lib
from .activations import add_bias2_nhwc_train, add_bias_nhwc, add_bias_nhwc_train, gelu, geglu, quick_gelu
from .attention import attention_reference, flash_attention, qkv_rope_attention
from .loss import cross_entropy, mse_loss
from .norms import group_norm, group_norm_cat, layer_norm
from .rope import apply_rotary_, rope_tables, rotary_reference

__all__ = [
    "_lib", "add_bias_nhwc", "add_bias_nhwc_train", "add_bias2_nhwc_train", "gelu", "geglu", "quick_gelu", "flash_attention", "qkv_rope_attention",
    "attention_reference", "cross_entropy", "mse_loss", "layer_norm", "group_norm", "group_norm_cat",
    "apply_rotary_", "rope_tables", "rotary_reference",
]
