"""Flash attention with softmax-P quant-dequant on MFMA (reference
``modelopt/torch/kernels/common/attention``: ``triton_fa.attention`` and the HF wrapper
``hf_triton_attention``).  The names of the reference are kept as aliases."""

from .flash_attention import LOG2E, attention
from .hf_attention import (
    attention_forward,
    triton_attention_forward,
    validate_attention_envelope,
    validate_triton_attention_envelope,
)

__all__ = [
    "LOG2E",
    "attention",
    "attention_forward",
    "triton_attention_forward",
    "validate_attention_envelope",
    "validate_triton_attention_envelope",
]
