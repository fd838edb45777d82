"""Quantization utilities (reductions, export-mode flag)."""

from .core_utils import *  # noqa: F403


def is_torch_export_mode() -> bool:
    """Reference: modelopt/torch/quantization/utils/core_utils.py (export-mode flag)."""
    try:
        import torch

        return torch.compiler.is_exporting()
    except Exception:  # noqa: BLE001
        return False
