"""Module replacement and wildcard quantizer configuration (reference: conversion.py:63-670)."""

from __future__ import annotations

import contextlib
import fnmatch
import functools
import re
from collections.abc import Callable
from typing import Any

import torch.nn as nn

from .config import QuantizeConfig, QuantizerAttributeConfig, normalize_quant_cfg_list
from .nn.modules.quant_module import QuantModule, QuantModuleRegistry
from .nn.modules.tensor_quantizer import SequentialQuantizer, TensorQuantizer, _AttributeItems
from .utils.names import is_quantized

__all__ = [
    "convert_to_quantized_model",
    "preserve_quantizer_attributes_context",
    "quantizer_state",
    "register",
    "replace_quant_module",
    "restore_quantizer_state",
    "set_quantizer_attribute",
    "set_quantizer_attributes_full",
    "set_quantizer_attributes_partial",
    "set_quantizer_by_cfg",
    "set_quantizer_by_cfg_context",
    "unregister",
]


def convert_to_quantized_model(model: nn.Module, config: QuantizeConfig | dict):
    """Insert quantizers and apply ``quant_cfg`` (reference :63-74)."""
    quant_cfg = config.get("quant_cfg", []) if isinstance(config, dict) else config.quant_cfg
    replace_quant_module(model)
    set_quantizer_by_cfg(model, quant_cfg)
    return model, {"quantizer_state": quantizer_state(model)}


def quantizer_state(model: nn.Module) -> dict[str, Any]:
    return {
        n: m.get_modelopt_state()
        for n, m in model.named_modules()
        if isinstance(m, (TensorQuantizer, SequentialQuantizer))
    }


def restore_quantizer_state(model: nn.Module, config, metadata: dict):
    """Restore quantizer properties + buffer shapes from ``metadata["quantizer_state"]``
    (reference :125-168): the saved and the model's quantizer sets must match; static-block
    quantizers are promoted before their state is applied (:103-108)."""
    from .nn.modules.tensor_quantizer import StaticBlockScaleQuantizer

    if "quantizer_state" not in metadata:
        return model
    state = metadata["quantizer_state"]
    current = quantizer_state(model).keys()
    unmatched, extra = state.keys() - current, current - state.keys()
    if unmatched:
        raise RuntimeError(f"Unmatched keys in quantizer state_dict: {unmatched}")
    if extra:
        raise RuntimeError(f"Extra keys in quantizer state_dict: {extra}")
    for name, module in model.named_modules():
        if isinstance(module, TensorQuantizer) and name in state:
            st = state[name]
            if (st.get("_is_static_block_scale_quantizer") or st.get("_is_nvfp4_static_quantizer")) and not isinstance(
                module, StaticBlockScaleQuantizer
            ):
                StaticBlockScaleQuantizer.from_tensor_quantizer(module)
            module.set_from_modelopt_state(st)
    for name, module in model.named_modules():
        if isinstance(module, QuantModule):
            module.modelopt_post_restore(name)
    return model


def replace_quant_module(model: nn.Module, version=None, registry=QuantModuleRegistry):
    """Recursively replace registered modules by their quantized versions (reference :214-242)."""
    from .plugins import register_custom_model_plugins_on_the_fly

    assert not is_quantized(model), "Model must not be quantized!"
    register_custom_model_plugins_on_the_fly(model)
    if type(model) in registry:
        model = registry.convert(model)
    _replace_quant_module(model, registry=registry)
    n = sum(isinstance(m, TensorQuantizer) for _, m in model.named_modules())
    print(f"Inserted {n} quantizers")


def _replace_quant_module(model: nn.Module, registry=QuantModuleRegistry):
    for name, child in model.named_children():
        if type(child) in registry:
            setattr(model, name, registry.convert(child))
        _replace_quant_module(getattr(model, name), registry=registry)


_FUSED_EXPERTS_QUANTIZER_LIST_RE = re.compile(r"(weight_quantizers?|input_quantizers?)\.\d+(?=$|\.)")


def _normalize_fused_experts_quantizer_name(name: str) -> str:
    """``...gate_up_proj_weight_quantizers.3`` -> ``...gate_up_proj_weight_quantizer`` (:322-341)."""
    return _FUSED_EXPERTS_QUANTIZER_LIST_RE.sub(lambda m: m.group(1).removesuffix("s"), name)


@functools.lru_cache(maxsize=4096)
def _wildcard_re(pattern: str):
    return re.compile(fnmatch.translate(pattern))


@functools.lru_cache(maxsize=65536)
def _normalized_name(name: str) -> str:
    return _normalize_fused_experts_quantizer_name(name)


def _quantizer_items(model: nn.Module):
    """The (name, quantizer) pairs of ``model``: the only modules a quant_cfg entry can match."""
    return [(n, m) for n, m in model.named_modules() if isinstance(m, (TensorQuantizer, SequentialQuantizer))]


def _match_quantizer(wildcard_or_filter_func, name, module, parent_class, full_model) -> bool:
    if not isinstance(module, (TensorQuantizer, SequentialQuantizer)):
        return False
    if isinstance(wildcard_or_filter_func, str):
        rx = _wildcard_re(wildcard_or_filter_func)
        normalized = _normalized_name(name)
        if not (rx.match(name) or (normalized != name and rx.match(normalized))):
            return False
    elif callable(wildcard_or_filter_func):
        if not wildcard_or_filter_func(name):
            return False
    else:
        raise NotImplementedError(f"Unsupported type {type(wildcard_or_filter_func)}")
    return parent_class is None or isinstance(
        full_model.get_submodule(".".join(name.split(".")[:-1])), parent_class
    )


def set_quantizer_by_cfg(quant_model: nn.Module, quant_cfg):
    """Apply an ordered quant_cfg list (reference :245-314): later entries win; an entry with
    ``cfg`` fully replaces the attributes, an ``enable``-only entry toggles."""
    qitems = [_quantizer_items(quant_model)]  # refreshed when a full entry swaps quantizer types
    for entry in normalize_quant_cfg_list(quant_cfg):
        name = entry["quantizer_name"]
        cfg = entry["cfg"]
        enable = entry["enable"]
        pc_name = entry.get("parent_class")
        if pc_name:
            try:
                parent_class = QuantModuleRegistry[pc_name]
            except KeyError:
                parent_class = None
                # a class with no quantized equivalent has no quantizers to match
                continue
        else:
            parent_class = None
        if cfg is None:
            set_quantizer_attributes_partial(quant_model, name, {"enable": enable}, parent_class, _items=qitems[0])
        else:
            if isinstance(cfg, QuantizerAttributeConfig):
                attributes = cfg.model_copy(update={"enable": enable})
            elif isinstance(cfg, dict):
                attributes = QuantizerAttributeConfig(**cfg, enable=enable)
            else:
                attributes = [
                    c.model_copy(update={"enable": enable})
                    if isinstance(c, QuantizerAttributeConfig)
                    else QuantizerAttributeConfig(**c, enable=enable)
                    for c in cfg
                ]
            if set_quantizer_attributes_full(quant_model, name, attributes, parent_class, _items=qitems[0]):
                qitems[0] = _quantizer_items(quant_model)


def set_quantizer_attributes_full(quant_model, wildcard_or_filter_func, attributes, parent_class=None,
                                  _items=None) -> bool:
    """Fully replace matched quantizers' attributes (reference :373-440).  Returns whether a
    quantizer module was swapped (TensorQuantizer <-> SequentialQuantizer)."""
    if not isinstance(attributes, (QuantizerAttributeConfig, list)):
        raise ValueError(f"Invalid type for attributes: {type(attributes)}")
    # validated once, applied to every matched quantizer
    applied = (
        [_AttributeItems(a.items()) for a in attributes]
        if isinstance(attributes, list)
        else _AttributeItems(attributes.items())
    )
    swapped = False
    for name, module in list(_items if _items is not None else quant_model.named_modules()):
        if not _match_quantizer(wildcard_or_filter_func, name, module, parent_class, quant_model):
            continue
        if isinstance(attributes, list):
            if not isinstance(module, SequentialQuantizer) or len(attributes) != len(module):
                parent = quant_model.get_submodule(name.rpartition(".")[0])
                module = SequentialQuantizer(*(TensorQuantizer() for _ in range(len(attributes))))
                setattr(parent, name.rpartition(".")[-1], module)
                swapped = True
            module.set_from_attribute_config(applied)
        else:
            if isinstance(module, SequentialQuantizer):
                parent = quant_model.get_submodule(name.rpartition(".")[0])
                module = TensorQuantizer()
                setattr(parent, name.rpartition(".")[-1], module)
                swapped = True
            module.set_from_attribute_config(applied)
    return swapped


def set_quantizer_attributes_partial(quant_model, wildcard_or_filter_func, partial: dict, parent_class=None,
                                     _items=None):
    """Update only the given attributes of matched quantizers (reference :443-505)."""
    for name, module in _items if _items is not None else quant_model.named_modules():
        if _match_quantizer(wildcard_or_filter_func, name, module, parent_class, quant_model):
            if isinstance(module, SequentialQuantizer):
                for q in module:
                    q.set_from_attribute_config(partial)
            else:
                module.set_from_attribute_config(partial)


def set_quantizer_attribute(quant_model, wildcard_or_filter_func, attribute, parent_class=None):
    """Legacy partial setter (reference :602-618)."""
    if isinstance(attribute, QuantizerAttributeConfig):
        attribute = {k: getattr(attribute, k) for k in attribute.model_fields_set}
    if isinstance(attribute, list):
        set_quantizer_attributes_full(quant_model, wildcard_or_filter_func, attribute, parent_class)
    else:
        set_quantizer_attributes_partial(quant_model, wildcard_or_filter_func, attribute, parent_class)


@contextlib.contextmanager
def set_quantizer_by_cfg_context(quant_model: nn.Module, quant_cfg):
    """Temporarily apply ``quant_cfg`` (enable-only entries), restoring the quantizers on exit
    (reference :568-600)."""
    entries = normalize_quant_cfg_list(quant_cfg)
    assert all(e["cfg"] is None for e in entries), "only enable/disable entries are supported"
    saved = {}
    for name, module in quant_model.named_modules():
        if isinstance(module, TensorQuantizer):
            saved[module] = module._disabled
    set_quantizer_by_cfg(quant_model, entries)
    try:
        yield
    finally:
        for module, disabled in saved.items():
            module._disabled = disabled


def register(original_cls: nn.Module, quantized_cls: nn.Module):
    """Register a custom (original -> quantized) pair (reference :620-662)."""
    assert issubclass(quantized_cls, QuantModule) or hasattr(quantized_cls, "_setup")
    QuantModuleRegistry.register({original_cls: original_cls.__name__})(quantized_cls)


def unregister(original_cls: nn.Module):
    QuantModuleRegistry.unregister(original_cls)


ReplaceFilter = Callable[[str], bool]


@contextlib.contextmanager
def preserve_quantizer_attributes_context(quant_model: nn.Module):
    """Restore every quantizer's properties (``get_modelopt_state(properties_only=True)``) and its
    TensorQuantizer / SequentialQuantizer type on exit -- parameters, buffers and calibrators are
    not copied (reference conversion.py:507-567).  A quantizer that a cfg change inside swapped
    for the other type is rebuilt in its original type first."""
    saved: dict[str, tuple] = {}
    for name, m in quant_model.named_modules():
        if isinstance(m, SequentialQuantizer):
            saved[name] = (SequentialQuantizer, [q.get_modelopt_state(properties_only=True) for q in m])
        elif isinstance(m, TensorQuantizer):
            saved[name] = (TensorQuantizer, m.get_modelopt_state(properties_only=True))
    try:
        yield
    finally:
        for name, m in list(quant_model.named_modules()):
            if name not in saved:
                continue
            kind, state = saved[name]
            parent_name, _, attr = name.rpartition(".")
            parent = quant_model.get_submodule(parent_name) if parent_name else quant_model
            if kind is SequentialQuantizer and not isinstance(m, SequentialQuantizer):
                m = SequentialQuantizer(*(TensorQuantizer() for _ in state))
                setattr(parent, attr, m)
                for q, st in zip(m, state):
                    q.set_from_modelopt_state(st, properties_only=True)
            elif kind is TensorQuantizer and not isinstance(m, TensorQuantizer):
                m = TensorQuantizer()
                setattr(parent, attr, m)
                m.set_from_modelopt_state(state, properties_only=True)
            elif kind is TensorQuantizer:
                m.set_from_modelopt_state(state, properties_only=True)
            else:  # still a SequentialQuantizer
                for q, st in zip(m, state):
                    q.set_from_modelopt_state(st, properties_only=True)

