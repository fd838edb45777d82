"""INT8 packed weights (reference qtensor/int8_tensor.py:30-124), the reference's expression on the
device."""

from __future__ import annotations

import torch

from ..utils.core_utils import convert_quantization_axis_to_reduce_axis
from .base_qtensor import BaseQuantizedTensor, true_div
from .fp8_tensor import _block_amax, _pad_blocks

__all__ = ["INT8QTensor"]


class INT8QTensor(BaseQuantizedTensor):
    @classmethod
    def quantize(cls, input: torch.Tensor, scales: torch.Tensor | None = None, axis=None, block_sizes=None):
        original = input
        block_sizes = {k: v for k, v in (block_sizes or {}).items() if isinstance(k, int)}
        if scales is None:
            if block_sizes:
                input = _pad_blocks(input, block_sizes)
                amax = _block_amax(input, block_sizes)
            else:
                red = convert_quantization_axis_to_reduce_axis(input, axis)
                amax = input.abs().amax() if red is None else input.abs().amax(dim=red, keepdim=True)
            scales = true_div(amax, 127.0)
        expanded = scales.clone()
        for dim, bs in block_sizes.items():
            expanded = expanded.repeat_interleave(bs, dim=dim)
        q = (input / expanded).round().clamp(-128, 127).to(torch.int8)
        return cls(original.shape, original.dtype, q), scales

    def dequantize(self, dtype: torch.dtype | None = None, **kwarg):
        dtype = dtype or self.metadata["dtype"]
        scales = kwarg["scale"]
        for dim, bs in {k: v for k, v in (kwarg.get("block_sizes") or {}).items() if isinstance(k, int)}.items():
            scales = scales.repeat_interleave(bs, dim=dim)
        q = self._quantized_data
        out = q.view(torch.int8).to(dtype) * scales.to(q.device).to(dtype)
        return out[tuple(slice(0, s) for s in self.metadata["shape"])]
