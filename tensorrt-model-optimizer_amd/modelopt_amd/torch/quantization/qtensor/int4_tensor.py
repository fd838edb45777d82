"""INT4 packed weights, two codes per byte (reference qtensor/int4_tensor.py:27-130): the reference's
CPU expression on the device (codes + 8, even element in the high nibble)."""

from __future__ import annotations

import math

import torch

from .base_qtensor import BaseQuantizedTensor

__all__ = ["INT4QTensor"]


class INT4QTensor(BaseQuantizedTensor):
    @staticmethod
    def _get_quant_maxbound(num_bits):
        return 2 ** (num_bits - 1) - 1

    @classmethod
    def quantize(cls, input: torch.Tensor, block_size: int):
        mb = cls._get_quant_maxbound(4)
        assert input.shape[-1] % 2 == 0, "Input tensor must have even number on last dimension."
        original = input
        flat = input.reshape(-1)
        pad = (-flat.numel()) % block_size
        if pad:
            flat = torch.nn.functional.pad(flat, (0, pad))
        blocks = flat.view(-1, block_size)
        amax = blocks.abs().amax(dim=-1, keepdim=True)
        scales = (mb / amax).view(blocks.shape[0], -1)  # Tensor.__rtruediv__: reciprocal(amax) * 7
        q = (blocks * scales).flatten().round().clamp(-(mb + 1), mb) + (mb + 1)
        q = q.to(torch.uint8)
        packed = (q[::2] << 4 | q[1::2]).reshape(*original.shape[:-1], -1)
        return cls(original.shape, flat.dtype, packed), scales

    def dequantize(self, dtype: torch.dtype | None = None, **kwarg):
        dtype = dtype or self.metadata["dtype"]
        scales = kwarg["scale"]
        bs = kwarg["block_sizes"][-1]
        mb = self._get_quant_maxbound(4)
        q = self._quantized_data
        hi = (q >> 4).to(torch.long) - (mb + 1)
        lo = (q & 0x0F).to(torch.long) - (mb + 1)
        s = scales.to(q.device).view(-1, 1)
        hi = (hi.view(-1, bs // 2) / s).flatten().unsqueeze(-1).transpose(0, 1)
        lo = (lo.view(-1, bs // 2) / s).flatten().unsqueeze(-1).transpose(0, 1)
        n = math.prod(self.metadata["shape"])
        return torch.stack([hi, lo], dim=-1).view(-1)[:n].reshape(self.metadata["shape"]).to(dtype)
