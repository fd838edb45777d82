"""``mtq.compress``: pack the weights of a quantized model into real-quantized QTensors
(reference quantization/compress.py:53-227).

Every QuantLinear whose weight quantizer matches the compress config gets ``fake_quant=False``
and its weight replaced by a ``QTensorWrapper`` (FP8 / INT8 / INT4 / NVFP4 / MXFP4 / MXFP8), the
scales kept as ``_scale`` / ``_double_scale`` buffers of the weight quantizer; the module becomes
a ``RealQuantLinear`` whose forward dequantises the packed weight (the reference's fallback when
no real-quant GEMM backend matches -- none is registered in this build).  The packing runs on the
MI355X export kernels where the format has one (qtensor/__init__.py).
"""

from __future__ import annotations

import fnmatch
import warnings
from typing import Any

import torch
import torch.nn as nn

from .conversion import set_quantizer_attributes_partial
from .nn.modules.quant_linear import _QuantLinear
from .qtensor import QTensorWrapper, pack_real_quantize_weight
from .utils.names import is_quantized_linear

__all__ = ["CompressConfig", "RealQuantLinear", "compress", "is_real_quantized"]


class CompressConfig(dict):
    """{"compress": {pattern: bool}, "quant_gemm": bool} (reference config.py:1620-1633)."""

    def __init__(self, compress: dict[str, bool] | None = None, quant_gemm: bool = True):
        super().__init__(compress=dict(compress) if compress is not None else {"*": True}, quant_gemm=quant_gemm)

    @property
    def compress(self) -> dict[str, bool]:
        return self["compress"]

    @property
    def quant_gemm(self) -> bool:
        return self["quant_gemm"]


class RealQuantLinear(_QuantLinear):
    """QuantLinear with a packed weight (reference nn/modules/quant_linear.py:196-300).  Without a
    real-quant GEMM the forward is the fake-quant one, whose weight quantizer dequantises."""

    list_of_scale_tensors = ["_scale", "_double_scale", "_scale_zeros"]
    allow_real_quant_gemm = True

    def forward(self, input, *args, **kwargs):
        if getattr(self, "_use_real_quant_gemm", False) and not self.__dict__.get("_warned_no_gemm"):
            warnings.warn(f"RealQuantLinear: No real-quant GEMM found: {type(self).__name__}.")
            self.__dict__["_warned_no_gemm"] = True
        return super().forward(input, *args, **kwargs)


def _to_real_quant_class(module: nn.Module) -> None:
    if isinstance(module, RealQuantLinear):
        return
    orig = module._original_cls
    module.__class__ = type(f"RealQuant{orig.__name__}", (RealQuantLinear, orig), {"_original_cls": orig})


def _as_config(config) -> CompressConfig:
    if config is None:
        return CompressConfig()
    if isinstance(config, CompressConfig):
        return config
    if isinstance(config, dict) and ("compress" in config or "quant_gemm" in config):
        return CompressConfig(config.get("compress"), config.get("quant_gemm", True))
    if isinstance(config, dict):
        return CompressConfig(config)
    raise TypeError(f"Invalid compress config {config!r}")


def compress_convert(model: nn.Module, config: CompressConfig, skip_real_quantize_weight: bool = False):
    """reference compress.py:53-133."""
    for _, module in model.named_modules():
        if is_quantized_linear(module) and isinstance(module, _QuantLinear):
            _to_real_quant_class(module)
    cfg = config.compress
    if "default" in cfg and isinstance(cfg["default"], bool):
        set_quantizer_attributes_partial(model, "*weight_quantizer*", {"fake_quant": not cfg["default"]})
    for pattern, to_compress in cfg.items():
        if pattern == "default":
            continue
        if not isinstance(to_compress, bool):
            raise ValueError(f"Invalid compression configuration: {to_compress}, expected a boolean as value.")
        set_quantizer_attributes_partial(
            model, lambda name, p=pattern: fnmatch.fnmatch(name, p) and "weight_quantizer" in name,
            {"fake_quant": not to_compress},
        )
    if not skip_real_quantize_weight:
        pack_real_quantize_weight(model)
    if any(isinstance(getattr(m, "weight", None), QTensorWrapper) for m in model.modules()):
        warnings.warn(
            "Real quantization has been applied to the model. This feature is still experimental, "
            "and some functionalities may not be supported."
        )
    for m in model.modules():
        if isinstance(m, RealQuantLinear):
            m._use_real_quant_gemm = bool(config.quant_gemm) and m.allow_real_quant_gemm
    metadata: dict[str, Any] = {"real_quantizer_state": {}, "q_tensor_state": {}}
    for name, m in model.named_modules():
        if isinstance(m, RealQuantLinear):
            metadata["real_quantizer_state"][name] = m.weight_quantizer.get_modelopt_state()
            if isinstance(m.weight, QTensorWrapper):
                metadata["q_tensor_state"][name] = m.weight.get_state()
    return model, metadata


def compress(model: nn.Module, config=None) -> None:
    """Compress the weights of a quantized model in place (reference compress.py:196-221)."""
    cfg = _as_config(config)
    with torch.no_grad():
        _, metadata = compress_convert(model, cfg)
    entry = model.__dict__.setdefault("_modelopt_amd_mode", {"config": {}})
    entry["compress"] = {"config": dict(cfg), "metadata": metadata}


def is_real_quantized(model: nn.Module) -> bool:
    return any(isinstance(m, RealQuantLinear) for m in model.modules())
