"""MXFP8 packed weights: E4M3 elements + E8M0 exponents per 32 (reference qtensor/mxfp8_tensor.py:26-262).
Packing on the HIP kernel mtq_export_mxfp8."""

from __future__ import annotations

import torch

from modelopt_amd._ext import ops as _ops

from .base_qtensor import BaseQuantizedTensor

__all__ = ["MXFP8QTensor"]


class MXFP8QTensor(BaseQuantizedTensor):
    E4M3_MAX = 448.0
    BLOCK_SIZE = 32
    SCALE_DTYPE = torch.uint8

    @classmethod
    def _e8m0_from_weight(cls, weight: torch.Tensor) -> torch.Tensor:
        """The reference's expression (reduce_block_amax, _compute_e8m0_exponent, :38-92) on the
        device, for the weight dtypes the HIP packer does not take (fp32): ceil(log2(amax / 448))
        clamped to [-127, 127], -127 where amax / 448 is not > 0, biased by 127."""
        nb = weight.shape[-1] // cls.BLOCK_SIZE
        amax = weight.reshape(*weight.shape[:-1], nb, cls.BLOCK_SIZE).abs().amax(dim=-1)
        descale = amax.float() / cls.E4M3_MAX
        lg = torch.where(descale > 0, torch.log2(descale), torch.tensor(-127.0, device=descale.device))
        return (torch.clamp(torch.ceil(lg), min=-127, max=127) + 127).to(cls.SCALE_DTYPE)

    @classmethod
    def get_weights_scaling_factor(cls, weight: torch.Tensor) -> torch.Tensor:
        assert weight.dim() >= 2, f"Weight must be at least 2D, got {weight.dim()}D"
        assert weight.shape[-1] % cls.BLOCK_SIZE == 0, (
            f"Weight inner dimension ({weight.shape[-1]}) must be divisible by MXFP8 block size ({cls.BLOCK_SIZE})")
        if weight.dtype in (torch.bfloat16, torch.float16):
            return _ops().export_mxfp8(weight)[1]
        return cls._e8m0_from_weight(weight)

    @classmethod
    def get_weights_scaling_factor_from_quantizer(cls, weight: torch.Tensor, weight_quantizer) -> torch.Tensor:
        """reference :98-138: the quantizer's ``_scale`` when compressed, else from the weight."""
        assert weight_quantizer.block_sizes[-1] == cls.BLOCK_SIZE, (
            f"MXFP8 requires block size {cls.BLOCK_SIZE}, got {weight_quantizer.block_sizes[-1]}"
        )
        expected = (*weight.shape[:-1], weight.shape[-1] // cls.BLOCK_SIZE)
        scale = getattr(weight_quantizer, "_scale", None)
        if scale is not None:
            assert scale.dtype == cls.SCALE_DTYPE and tuple(scale.shape) == expected
            return scale
        return cls.get_weights_scaling_factor(weight)

    @classmethod
    def quantize_with_scale(cls, weight: torch.Tensor, weights_scaling_factor: torch.Tensor) -> torch.Tensor:
        """e4m3(clamp(w * 2^(127 - s), +-448)) with a given E8M0 scale (reference :140-161)."""
        assert weights_scaling_factor.dtype == cls.SCALE_DTYPE
        nb = weight.shape[-1] // cls.BLOCK_SIZE
        f = torch.exp2(127 - weights_scaling_factor.float()).unsqueeze(-1)
        w = weight.view(*weight.shape[:-1], nb, cls.BLOCK_SIZE) * f
        return w.clamp(-cls.E4M3_MAX, cls.E4M3_MAX).to(torch.float8_e4m3fn).view(weight.shape)

    @classmethod
    def quantize(cls, input: torch.Tensor, weights_scaling_factor: torch.Tensor | None = None):
        if weights_scaling_factor is None and input.shape[-1] % cls.BLOCK_SIZE == 0:
            if input.dtype in (torch.bfloat16, torch.float16):
                q, s = _ops().export_mxfp8(input)
                return cls(input.shape, input.dtype, q), s
            weights_scaling_factor = cls._e8m0_from_weight(input)
        assert weights_scaling_factor is not None, "MXFP8: last dim must be a multiple of 32"
        return cls(input.shape, input.dtype, cls.quantize_with_scale(input, weights_scaling_factor)), weights_scaling_factor

    def dequantize(self, dtype: torch.dtype | None = None, **kwargs):
        e8m0 = kwargs["scale"]
        dtype = dtype or self.metadata["dtype"]
        q = self._quantized_data.float()
        nb = q.shape[-1] // self.BLOCK_SIZE
        out = q.view(*q.shape[:-1], nb, self.BLOCK_SIZE) * torch.exp2(e8m0.to(q.device).float() - 127).unsqueeze(-1)
        return out.view(q.shape)[..., : self.metadata["shape"][-1]].to(dtype)
