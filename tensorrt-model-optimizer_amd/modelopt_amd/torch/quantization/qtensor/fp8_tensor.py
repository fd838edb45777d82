"""FP8 (E4M3) packed weights (reference qtensor/fp8_tensor.py:31-151)."""

from __future__ import annotations

import math

import torch

from modelopt_amd._ext import ops as _ops

from ..utils.core_utils import convert_quantization_axis_to_reduce_axis
from .base_qtensor import BaseQuantizedTensor, true_div

__all__ = ["FP8QTensor"]


def _pad_blocks(x, block_sizes):
    for dim, bs in block_sizes.items():
        if not isinstance(dim, int):
            continue
        d = dim if dim >= 0 else x.dim() + dim
        pad = (-x.shape[d]) % bs
        if pad:
            p = [0, 0] * (x.dim() - d - 1) + [0, pad]
            x = torch.nn.functional.pad(x, p)
    return x


def _block_amax(x, block_sizes):
    """reduce_block_amax: |x| max over each block (kept dims collapsed to the block grid)."""
    shape, view = [], []
    for d, s in enumerate(x.shape):
        bs = block_sizes.get(d, block_sizes.get(d - x.dim()))
        if bs:
            view += [s // bs, bs]
            shape.append(len(view) - 1)
        else:
            view.append(s)
    return x.reshape(view).abs().amax(dim=shape)


class FP8QTensor(BaseQuantizedTensor):
    @classmethod
    def quantize(cls, input: torch.Tensor, scales: torch.Tensor | None = None, axis=None, block_sizes=None):
        """(FP8QTensor, scales): ``(input / scales).to(float8_e4m3fn)``; scales = amax / 448 when
        not given.  The per-tensor case runs the HIP packer (the bf16 quotient rounded to the
        weight dtype first, as torch's bf16 / 0-d division does); per-channel and block scales
        evaluate the reference expression on the device."""
        original = input
        block_sizes = {k: v for k, v in (block_sizes or {}).items() if isinstance(k, int)}
        if block_sizes:
            input = _pad_blocks(input, block_sizes)
        if scales is None:
            if block_sizes:
                amax = _block_amax(input, block_sizes)
            else:
                red = convert_quantization_axis_to_reduce_axis(input, axis)
                amax = input.abs().amax() if red is None else input.abs().amax(dim=red, keepdim=True)
            scales = true_div(amax, 448.0)
        if scales.numel() == 1 and not block_sizes and input.is_cuda and input.dtype in (torch.bfloat16, torch.float16):
            q = _ops().export_fp8(input, scales.reshape(()), False, scales.dtype == input.dtype or scales.dim() == 0)
            return cls(original.shape, original.dtype, q), scales
        expected = list(input.shape)
        expanded = scales.clone()
        if block_sizes:
            for dim, bs in block_sizes.items():
                d = dim if dim >= 0 else input.dim() + dim
                expected[d] = input.shape[d] // bs
            if scales.shape != tuple(expected) and scales.numel() == math.prod(expected):
                scales = scales.reshape(expected)
                expanded = expanded.reshape(expected)
            assert scales.shape == tuple(expected), (
                f"Mismatch in expected scale shape: {scales.shape} vs {tuple(expected)}")
            bs2 = {(d if d >= 0 else input.dim() + d): b for d, b in block_sizes.items()}
            vec = 16 // original.element_size()
            if (original.dim() == 2 and set(bs2) == {0, 1} and original.is_cuda
                    and original.dtype in (torch.bfloat16, torch.float16, torch.float32)
                    and scales.dtype in (torch.float32, original.dtype)
                    and original.shape[1] % vec == 0 and bs2[1] % vec == 0
                    and original.data_ptr() % 16 == 0):
                # the 2D-block packer (one pass; the expression below materialises the expanded
                # scales and the fp32 quotient): same quotient dtype and RNE convert
                q = _ops().export_fp8_block2d(original, scales, bs2[0], bs2[1])
                return cls(original.shape, original.dtype, q), scales
            for dim, bs in block_sizes.items():
                expanded = expanded.repeat_interleave(bs, dim=dim)
        q = (input / expanded).to(torch.float8_e4m3fn)
        q = q[tuple(slice(0, s) for s in original.shape)]
        return cls(original.shape, original.dtype, q), scales

    def dequantize(self, dtype: torch.dtype | None = None, **kwarg):
        dtype = dtype or self.metadata["dtype"]
        scales = kwarg["scale"]
        block_sizes = {k: v for k, v in (kwarg.get("block_sizes") or {}).items() if isinstance(k, int)}
        q = self._quantized_data
        if block_sizes:
            q = _pad_blocks(q.view(torch.uint8), block_sizes).view(torch.float8_e4m3fn)
            for dim, bs in block_sizes.items():
                scales = scales.repeat_interleave(bs, dim=dim)
        scales = scales.to(q.device)
        return (q.to(dtype) * scales.to(dtype))[tuple(slice(0, s) for s in self.metadata["shape"])]
