"""Base real-quantized tensor + the nn.Parameter wrapper (reference qtensor/base_qtensor.py:34-242)."""

from __future__ import annotations

import torch

__all__ = ["BaseQuantizedTensor", "QTensorWrapper", "pack_real_quantize_weight", "true_div"]


def true_div(t: torch.Tensor, c: float) -> torch.Tensor:
    """``t / c`` for a Python scalar ``c`` as the reference's CPU/CUDA torch computes it: an IEEE
    division in t's dtype.  torch on ROCm turns a division by a host scalar into a multiply by its
    reciprocal (1 ulp apart), so the divisor becomes a 0-d device tensor of t's dtype."""
    return torch.div(t, torch.tensor(c, dtype=t.dtype, device=t.device))


class BaseQuantizedTensor:
    """Packed data + the original shape / dtype (reference :34-86)."""

    _quantized_data: torch.Tensor

    def __init__(self, original_shape: torch.Size, original_dtype: torch.dtype, quantized_data: torch.Tensor):
        self.metadata = {"shape": original_shape, "dtype": original_dtype}
        self._quantized_data = quantized_data

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        torch.serialization.add_safe_globals([cls])

    @classmethod
    def quantize(cls, input: torch.Tensor, block_size: int):
        raise NotImplementedError("This method must be implemented by subclasses.")

    def dequantize(self, dtype: torch.dtype | None = None, **kwarg):
        raise NotImplementedError("This method must be implemented by subclasses.")


class QTensorWrapper(torch.nn.Parameter):
    """nn.Parameter holding the packed data, with the QTensor class / shape / dtype in
    ``metadata`` (reference :89-146)."""

    def __new__(cls, qtensor: BaseQuantizedTensor | torch.Tensor, metadata: dict | None = None):
        data = qtensor._quantized_data if isinstance(qtensor, BaseQuantizedTensor) else qtensor
        instance = super().__new__(cls, data, requires_grad=False)
        if metadata is None:
            instance.metadata = dict(qtensor.metadata)
            instance.metadata["qtensor_class"] = qtensor.__class__
        else:
            assert all(k in metadata for k in ("qtensor_class", "shape", "dtype")), f"metadata: {metadata}"
            instance.metadata = metadata
        return instance

    def dim(self):
        return len(self.metadata["shape"])

    def to(self, *args, **kwargs):
        device, dtype, *_ = torch._C._nn._parse_to(*args, **kwargs)
        if device:
            self.data = self.data.to(device=device)
        dtype = dtype or self.metadata["dtype"]
        return QTensorWrapper(self.metadata["qtensor_class"](self.metadata["shape"], dtype, self.data))

    def get_qtensor(self):
        return self.metadata["qtensor_class"](self.metadata["shape"], self.metadata["dtype"], self.data)

    def get_state(self):
        return {
            "metadata": self.metadata,
            "quantized_data.shape": self.data.shape,
            "quantized_data.dtype": self.data.dtype,
        }


def pack_real_quantize_weight(module, force_quantize: bool = False):
    """Replace every enabled, non-fake weight quantizer's weight by its QTensorWrapper
    (reference :204-238)."""
    from ..nn.modules.tensor_quantizer import SequentialQuantizer

    def _compress(m) -> bool:
        w = getattr(m, "weight", None)
        if not hasattr(m, "weight") or w is None or w.is_meta:
            return False
        wq = getattr(m, "weight_quantizer", None)
        if wq is None:
            return False
        if isinstance(wq, SequentialQuantizer):
            wq = wq[0]
        if wq.is_enabled and not wq._fake_quant and w.element_size() > 1:
            if force_quantize:
                wq._dequantize = False
            m.weight = QTensorWrapper(wq(w))
            return True
        return False

    with torch.no_grad():
        for name, m in module.named_modules():
            if name != "":
                _compress(m)


torch.serialization.add_safe_globals([QTensorWrapper])
