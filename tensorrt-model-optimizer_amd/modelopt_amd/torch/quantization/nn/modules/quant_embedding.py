"""Quantized Embedding (reference: nn/modules/quant_embedding.py).

The lookup indices cannot be fake-quantized, so ``input_quantizer`` is a permanently disabled
placeholder (kept for introspection by config matching and export, whose exclude list names the
embedding); the table (``weight_quantizer``) and the lookup output (``output_quantizer``) are
quantizable.  Every default config disables ``nn.Embedding`` quantizers (``parent_class`` entry).
"""

import torch.nn as nn

from ... import tensor_quant
from .quant_module import QuantLinearConvBase, QuantModuleRegistry
from .tensor_quantizer import TensorQuantizer

__all__ = ["QuantEmbedding"]


class HardDisabledTensorQuantizer(TensorQuantizer):
    """A quantizer that stays disabled whatever a config asks (reference tensor_quantizer.py)."""

    def enable(self):
        self.disable()

    def set_from_attribute_config(self, attribute_cfg):
        super().set_from_attribute_config(attribute_cfg)
        self.disable()


@QuantModuleRegistry.register({nn.Embedding: "nn.Embedding"})
class _QuantEmbedding(QuantLinearConvBase):
    default_quant_desc_weight = tensor_quant.QUANT_DESC_8BIT_PER_TENSOR

    def _setup(self):
        super()._setup()
        self._register_temp_attribute("input_quantizer", HardDisabledTensorQuantizer())
        self.input_quantizer.disable()

    def forward(self, input, *args, **kwargs):
        with self.quantize_weight():
            out = self._original_cls.forward(self, input, *args, **kwargs)
        return self.output_quantizer(out)


QuantEmbedding = _QuantEmbedding
