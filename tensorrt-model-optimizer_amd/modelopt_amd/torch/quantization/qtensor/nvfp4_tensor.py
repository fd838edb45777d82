"""NVFP4 packed weights: E2M1 codes, E4M3 per-16 scales, fp32 global scale (reference
qtensor/nvfp4_tensor.py:52-407).  Scales from the export helpers, packing on mtq_export_nvfp4."""

from __future__ import annotations

import torch

from modelopt_amd._ext import ops as _ops

from .base_qtensor import BaseQuantizedTensor

__all__ = ["NVFP4QTensor"]

_E2M1 = [0, 0.5, 1, 1.5, 2, 3, 4, 6, 0, -0.5, -1, -1.5, -2, -3, -4, -6]


class NVFP4QTensor(BaseQuantizedTensor):
    @classmethod
    def get_weights_scaling_factor_2_from_quantizer(cls, weight_quantizer):
        from ...export.quant_utils import nvfp4_weights_scaling_factor_2_from_quantizer

        return nvfp4_weights_scaling_factor_2_from_quantizer(weight_quantizer)

    @classmethod
    def get_weights_scaling_factor_2(cls, input: torch.Tensor):
        from ...export.quant_utils import _div

        return _div(input.abs().amax().float(), 6.0 * 448.0)

    @classmethod
    def quantize(cls, input: torch.Tensor, block_size: int, weights_scaling_factor=None,
                 weights_scaling_factor_2=None, keep_high_precision: bool = False, try_tensorrt: bool = False):
        from ...export.quant_utils import nvfp4_weights_scaling_factor

        if weights_scaling_factor_2 is None:
            weights_scaling_factor_2 = cls.get_weights_scaling_factor_2(input)
        if weights_scaling_factor is None:
            weights_scaling_factor = nvfp4_weights_scaling_factor(input, block_size, weights_scaling_factor_2)
        q = _ops().export_nvfp4(input, weights_scaling_factor.to(torch.float32), weights_scaling_factor_2)
        return cls(input.shape, input.dtype, q), weights_scaling_factor, weights_scaling_factor_2

    def dequantize(self, dtype: torch.dtype | None = None, fast=False, **kwarg):
        dtype = dtype or self.metadata["dtype"]
        x = self._quantized_data
        scale = kwarg["scale"]
        s = scale.to(torch.float32) if scale.dtype == torch.float8_e4m3fn else scale
        per_block = s.to(x.device) * kwarg["double_scale"].to(x.device)
        shape = list(x.shape)
        shape[-1] *= 2
        codes = torch.empty(shape, dtype=torch.uint8, device=x.device)
        codes[..., 1::2] = x >> 4
        codes[..., 0::2] = x & 0x0F
        vals = torch.tensor(_E2M1, dtype=torch.float32, device=x.device)[codes.long().reshape(-1)].reshape(shape)
        bs = kwarg["block_sizes"][-1]
        out = vals.view(*shape[:-1], -1, bs) * per_block.unsqueeze(-1)
        return out.reshape(self.metadata["shape"]).to(dtype)
