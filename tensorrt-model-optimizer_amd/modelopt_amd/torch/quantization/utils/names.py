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


def representative_weight_quantizer(module: nn.Module, weight_name: str = "weight"):
    """The weight quantizer of ``weight_name``: singular ``<name>_weight_quantizer``, or the first
    of a fused-experts plural ``<name>_weight_quantizers`` ModuleList (reference core_utils.py:215)."""
    from ..nn.modules.tensor_quantizer import SequentialQuantizer, TensorQuantizer

    q = module._modules.get(quantizer_attr_names(weight_name).weight_quantizer)
    if isinstance(q, (TensorQuantizer, SequentialQuantizer)):
        return q
    plural = module._modules.get(quantizer_attr_names(weight_name).weight_quantizer + "s")
    if isinstance(plural, nn.ModuleList) and len(plural) > 0:
        first = plural[0]
        if isinstance(first, (TensorQuantizer, SequentialQuantizer)):
            return first
    return None


def weight_attr_names(module: nn.Module):
    """Names of the quantized weight parameters of a converted module (non-recursive)."""
    for name, p in module._parameters.items():
        if p is None:
            continue
        if representative_weight_quantizer(module, name) is not None:
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
