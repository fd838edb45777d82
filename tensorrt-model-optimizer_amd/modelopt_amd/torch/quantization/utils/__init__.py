"""Quantization utilities (reductions, names, export-mode flag)."""

from .core_utils import *  # noqa: F403
from .names import (  # noqa: F401
    QuantizerAttrNames,
    is_quantized,
    is_quantized_linear,
    quantizer_attr_names,
    weight_attr_names,
)


def is_torch_export_mode() -> bool:
    try:
        import torch

        return torch.compiler.is_exporting()
    except Exception:  # noqa: BLE001
        return False
