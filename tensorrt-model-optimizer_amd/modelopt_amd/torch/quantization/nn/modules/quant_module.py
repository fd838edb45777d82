"""Quantized-module wrappers (reference: nn/modules/quant_module.py:41-278).

The reference builds these on its DynamicModule framework (modelopt/torch/opt/dynamic.py): an
existing module's class is swapped in place for a generated subclass and a "dynamic attribute"
makes ``self.weight`` return the fake-quantised weight inside the original ``forward``.  Here the
same contract is implemented directly: ``QuantModuleRegistry.convert`` swaps ``module.__class__``
to ``type("Quant" + cls, (quant_cls, cls))`` (parameters and buffers untouched) and calls
``_setup``; ``QuantLinearConvBase.__getattr__`` intercepts ``weight`` while
``_enable_weight_quantization`` is set (opt/dynamic.py:767-787).
"""

from __future__ import annotations

import contextlib
import warnings
from typing import Any

import torch
import torch.nn as nn

from modelopt_amd.torch.utils.distributed import ParallelState

from ...calib.max import quantizer_call_is_noop
from ...tensor_quant import QUANT_DESC_8BIT_PER_TENSOR
from .tensor_quantizer import SequentialQuantizer, TensorQuantizer

__all__ = ["QuantInputBase", "QuantLinearConvBase", "QuantModule", "QuantModuleRegistry"]


class _QuantModuleRegistry:
    """original nn class -> quantized wrapper class, with by-name lookup ("nn.Linear")."""

    def __init__(self):
        self._by_cls: dict[type, type] = {}
        self._names: dict[str, type] = {}
        self._generated: dict[tuple[type, type], type] = {}

    def register(self, cls_to_key: dict[type, str]):
        def decorator(quant_cls):
            for cls, key in cls_to_key.items():
                self._by_cls[cls] = quant_cls
                self._names[key] = cls
            return quant_cls

        return decorator

    def unregister(self, cls: type):
        self._by_cls.pop(cls, None)
        for k in [k for k, v in self._names.items() if v is cls]:
            self._names.pop(k)

    def __contains__(self, cls) -> bool:
        if isinstance(cls, str):
            return cls in self._names
        return cls in self._by_cls

    def __getitem__(self, key):
        """Registry lookup by key ("nn.Linear") or original class -> the *quantized* class."""
        cls = self._names[key] if isinstance(key, str) else key
        if cls not in self._by_cls:
            raise KeyError(key)
        return self._dynamic_cls(cls, self._by_cls[cls])

    def get(self, key, default=None):
        try:
            return self[key]
        except KeyError:
            return default

    def _dynamic_cls(self, orig: type, quant_cls: type) -> type:
        k = (orig, quant_cls)
        if k not in self._generated:
            self._generated[k] = type(
                f"Quant{orig.__name__}", (quant_cls, orig), {"_original_cls": orig}
            )
        return self._generated[k]

    def convert(self, module: nn.Module, **setup_kwargs) -> nn.Module:
        orig = type(module)
        if orig not in self._by_cls:
            raise KeyError(f"{orig} is not registered for quantization")
        module.__class__ = self._dynamic_cls(orig, self._by_cls[orig])
        module._setup(**setup_kwargs)
        if module.parallel_state is None:
            module._initialize_parallel_state()
        return module


QuantModuleRegistry = _QuantModuleRegistry()

# data-parallel group newly converted modules sync their amax over (None = world, -1 = none);
# layer-sharded calibration (sharded.py) switches it to -1 while it runs
_DEFAULT_DP_GROUP = None


class QuantModule(nn.Module):
    """Base class of quantized modules (reference :41)."""

    _original_cls: type = nn.Module

    def _setup(self):
        pass

    @classmethod
    def convert(cls, module: nn.Module, **setup_kwargs) -> "QuantModule":
        return QuantModuleRegistry.convert(module, **setup_kwargs)

    def _register_temp_attribute(self, name: str, value: Any):
        setattr(self, name, value)

    @property
    def parallel_state(self) -> ParallelState | None:
        return self.__dict__.get("_parallel_state", None)

    @parallel_state.setter
    def parallel_state(self, parallel_state: ParallelState):
        assert isinstance(parallel_state, ParallelState), "parallel_state must be a ParallelState object!"
        self.__dict__["_parallel_state"] = parallel_state

    def _initialize_parallel_state(self):
        self.parallel_state = ParallelState(data_parallel_group=_DEFAULT_DP_GROUP)

    def iter_weights_for_calibration(self):
        """Yield ``(weight, weight_quantizer)`` pairs for weight-only calibration."""
        from ...utils.names import quantizer_attr_names, weight_attr_names

        for weight_name in weight_attr_names(self):
            yield self._parameters_or_attr(weight_name), getattr(
                self, quantizer_attr_names(weight_name).weight_quantizer
            )

    def _parameters_or_attr(self, name):
        p = self._parameters.get(name)
        return p if p is not None else getattr(self, name)

    @staticmethod
    @torch.no_grad()
    def _fold_weight_quantizer(quantizer: TensorQuantizer, weights, keep_attrs: bool = False):
        if not quantizer.fake_quant:
            return
        for weight in weights:
            weight.data.copy_(quantizer(weight.float().contiguous()).to(weight.dtype))
        quantizer.disable()
        if keep_attrs and hasattr(quantizer, "_pre_quant_scale"):
            quantizer._enable_pre_quant_scale = False
        elif not keep_attrs:
            for attr in ("_pre_quant_scale", "_amax"):
                if hasattr(quantizer, attr):
                    delattr(quantizer, attr)

    def fold_weight(self, keep_attrs: bool = False):
        """Bake each fake-quant weight quantizer into its weight (reference :176-201)."""
        for name in list(self._modules):
            attr = self._modules[name]
            if name.endswith("weight_quantizer") and isinstance(attr, TensorQuantizer) and attr.fake_quant:
                weight_name = name[: -len("_quantizer")] if name != "weight_quantizer" else "weight"
                weight = self._parameters.get(weight_name)
                if weight is None:
                    weight = getattr(self, weight_name, None)
                if isinstance(weight, torch.Tensor):
                    self._fold_weight_quantizer(attr, (weight,), keep_attrs)

    def modelopt_post_restore(self, prefix: str = ""):
        """Move restored quantizer buffers to the device of the module's own parameters
        (reference quant_module.py:92-121): restored buffers are created on the CPU."""
        device = None
        for name, t in self.state_dict().items():
            parent = self.get_submodule(name.rsplit(".", 1)[0]) if "." in name else self
            if not isinstance(parent, TensorQuantizer):
                device = t.device
                break
        if device is None:
            warnings.warn(
                f"Could not identify the device for TensorQuantizer states of {prefix}. "
                "Please move the model to the right device now. This can be done by calling "
                "`model.to(device)`."
            )
            return
        for module in self.modules():
            if isinstance(module, TensorQuantizer):
                module.to(device)

    def export(self) -> nn.Module:
        """Drop the quantizers and restore the original class (the DynamicModule 'export')."""
        for name in [n for n, m in self._modules.items() if isinstance(m, (TensorQuantizer, SequentialQuantizer))]:
            delattr(self, name)
        self.__class__ = self._original_cls
        return self


class QuantInputBase(QuantModule):
    """Quantize the input (and optionally the output) around the original forward (:200-235)."""

    input_quantizer: TensorQuantizer
    output_quantizer: TensorQuantizer
    default_quant_desc_input = QUANT_DESC_8BIT_PER_TENSOR
    default_quant_desc_output = QUANT_DESC_8BIT_PER_TENSOR

    def forward(self, input, *args, **kwargs):
        input = self.input_quantizer(input)
        output = self._original_cls.forward(self, input, *args, **kwargs)
        if isinstance(output, tuple):
            return (self.output_quantizer(output[0]), *output[1:])
        return self.output_quantizer(output)

    def _setup(self):
        self._register_temp_attribute("input_quantizer", TensorQuantizer(self.default_quant_desc_input))
        self._register_temp_attribute("output_quantizer", TensorQuantizer(self.default_quant_desc_output))
        self.output_quantizer.disable()


class QuantLinearConvBase(QuantInputBase):
    """Quantize input and weight (reference :238-278)."""

    weight_quantizer: TensorQuantizer | SequentialQuantizer
    default_quant_desc_weight = QUANT_DESC_8BIT_PER_TENSOR

    @contextlib.contextmanager
    def quantize_weight(self):
        self.__dict__["_enable_weight_quantization"] = True
        try:
            yield
        finally:
            self.__dict__["_enable_weight_quantization"] = False

    def __getattr__(self, name):
        attr = super().__getattr__(name)
        if name == "weight" and self.__dict__.get("_enable_weight_quantization", False):
            wq = self._modules["weight_quantizer"]
            if type(wq) is TensorQuantizer and quantizer_call_is_noop(wq, attr):
                return attr  # max calibration: this weight version is already collected
            return wq(attr)
        return attr

    def forward(self, input, *args, **kwargs):
        with self.quantize_weight():
            return super().forward(input, *args, **kwargs)

    def _setup(self):
        super()._setup()
        self._register_temp_attribute("weight_quantizer", TensorQuantizer(self.default_quant_desc_weight))
        self.__dict__["_enable_weight_quantization"] = False

