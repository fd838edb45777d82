"""Quantized Linear (reference: nn/modules/quant_linear.py:38-53)."""

import torch.nn as nn

from ... import tensor_quant
from .quant_module import QuantLinearConvBase, QuantModuleRegistry

__all__ = ["Linear", "QuantLinear"]


@QuantModuleRegistry.register({nn.Linear: "nn.Linear"})
class _QuantLinear(QuantLinearConvBase):
    """Quantized base class for nn.Linear type classes: weight per-row INT8 by default."""

    default_quant_desc_weight = tensor_quant.QUANT_DESC_8BIT_LINEAR_WEIGHT_PER_ROW

    @staticmethod
    def quantized_linear_fn(package, func_name, self, input, weight, *args, **kwargs):
        """Quantized version of a generic linear functional (reference :44-53)."""
        output = getattr(package, func_name)(
            self.input_quantizer(input), self.weight_quantizer(weight), *args, **kwargs
        )
        return self.output_quantizer(output)


class QuantLinear(nn.Linear):
    """``nn.Linear`` that is born quantized (legacy constructor form, reference :56-61).  The
    class-level ``default_quant_desc_input`` / ``default_quant_desc_weight`` apply when no
    descriptor is passed (reference tests/unit/torch/quantization/test_quant_linear.py:199-222)."""

    default_quant_desc_input = tensor_quant.QUANT_DESC_8BIT_PER_TENSOR
    default_quant_desc_weight = tensor_quant.QUANT_DESC_8BIT_LINEAR_WEIGHT_PER_ROW

    def __new__(cls, *args, quant_desc_input=None, quant_desc_weight=None, **kwargs):
        m = nn.Linear(*args, **kwargs)
        QuantModuleRegistry.convert(m)
        m.input_quantizer.set_from_attribute_config(
            cls.default_quant_desc_input if quant_desc_input is None else quant_desc_input
        )
        m.weight_quantizer.set_from_attribute_config(
            cls.default_quant_desc_weight if quant_desc_weight is None else quant_desc_weight
        )
        return m


Linear = QuantLinear
