"""MXFP4 packed weights: E2M1 codes + E8M0 block exponents (reference qtensor/mxfp4_tensor.py:22-144).
Packing on the HIP export kernel (mtq_export_mxfp4, bit-exact with the reference)."""

from __future__ import annotations

import torch

from modelopt_amd._ext import ops as _ops

from .base_qtensor import BaseQuantizedTensor

__all__ = ["MXFP4QTensor"]


class MXFP4QTensor(BaseQuantizedTensor):
    E2M1_max = 6.0
    E2M1_values = [0, 0.5, 1, 1.5, 2, 3, 4, 6]
    E2M1_bounds = torch.tensor([0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5])

    @classmethod
    def quantize(cls, input: torch.Tensor, block_size: int | None):
        block_size = block_size or 32
        q, e8m0 = _ops().export_mxfp4(input, block_size)
        return cls(input.shape, input.dtype, q), e8m0

    def dequantize(self, dtype: torch.dtype | None = None, **kwarg):
        e8m0 = kwarg["scale"]
        block_size = kwarg["block_sizes"][-1]
        dtype = dtype or self.metadata["dtype"]
        x = self._quantized_data
        shape = list(x.shape)
        shape[-1] *= 2
        codes = torch.zeros(shape, dtype=torch.uint8, device=x.device)
        codes[..., 0::2] = x & 0x0F
        codes[..., 1::2] = (x >> 4) & 0x0F
        sign = 1 - 2 * ((codes & 0b1000) >> 3).to(torch.float32)
        values = torch.tensor(self.E2M1_values, device=x.device)
        xf = values[(codes & 0b0111).to(torch.long).reshape(-1)].reshape(codes.shape)
        xf = (sign * xf).reshape(-1, block_size) * torch.exp2(e8m0.to(x.device).float() - 127).reshape(-1, 1)
        return xf.reshape(codes.shape).to(dtype)
