"""Abstract calibrator (reference: modelopt/torch/quantization/calib/calibrator.py:25-75)."""

from typing import Any

import torch

__all__ = ["_Calibrator"]


class _Calibrator:
    """Base of calibrators: ``collect`` tensors, ``compute_amax``, ``reset``."""

    def __init__(self, num_bits=8, axis=None, unsigned=False):
        self._num_bits = num_bits
        self._axis = axis
        self._unsigned = unsigned

    def __init_subclass__(cls, **kwargs: Any) -> None:
        super().__init_subclass__(**kwargs)
        torch.serialization.add_safe_globals([cls])

    def collect(self, x):
        raise NotImplementedError

    def reset(self):
        raise NotImplementedError

    def compute_amax(self, *args, **kwargs):
        raise NotImplementedError

    def __repr__(self):
        return f"num_bits={self._num_bits} axis={self._axis} unsigned={self._unsigned}"
