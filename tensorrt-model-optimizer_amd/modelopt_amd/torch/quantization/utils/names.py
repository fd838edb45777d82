"""Weight / quantizer attribute-name helpers (reference: utils/core_utils.py:246-335)."""

from __future__ import annotations

from typing import NamedTuple

import torch.nn as nn


class QuantizerAttrNames(NamedTuple):
    weight_quantizer: str
    input_quantizer: str
    output_quantizer: str
    weight_scale: str
    weight_scale_2: str
    input_scale: str
    output_scale: str


def quantizer_attr_names(weight_name: str = "weight") -> QuantizerAttrNames:
    prefix = f"{weight_name}_" if weight_name != "weight" else ""
    return QuantizerAttrNames(
        weight_quantizer=f"{prefix}weight_quantizer",
        input_quantizer=f"{prefix}input_quantizer",
        output_quantizer=f"{prefix}output_quantizer",
        weight_scale=f"{prefix}weight_scale",
        weight_scale_2=f"{prefix}weight_scale_2",
        input_scale=f"{prefix}input_scale",
        output_scale=f"{prefix}output_scale",
    )


def weight_attr_names(module: nn.Module):
    """Names of the quantized weight parameters of a converted module (non-recursive)."""
    from ..nn.modules.tensor_quantizer import SequentialQuantizer, TensorQuantizer

    for name, p in module._parameters.items():
        if p is None:
            continue
        q = module._modules.get(quantizer_attr_names(name).weight_quantizer)
        if isinstance(q, (TensorQuantizer, SequentialQuantizer)):
            yield name


def is_quantized(module) -> bool:
    from ..nn.modules.tensor_quantizer import TensorQuantizer

    return any(isinstance(m, TensorQuantizer) for m in module.modules())


def is_quantized_linear(module) -> bool:
    """A QuantModule with input+weight quantizers and a 2-D weight (reference :317-335)."""
    from ..nn.modules.quant_module import QuantModule
    from ..nn.modules.tensor_quantizer import SequentialQuantizer, TensorQuantizer

    return (
        isinstance(module, QuantModule)
        and isinstance(getattr(module, "input_quantizer", None), TensorQuantizer)
        and isinstance(getattr(module, "weight_quantizer", None), (TensorQuantizer, SequentialQuantizer))
        and isinstance(module._parameters.get("weight"), nn.Parameter)
        and module._parameters["weight"].dim() == 2
        and not isinstance(module, nn.Embedding)
    )
