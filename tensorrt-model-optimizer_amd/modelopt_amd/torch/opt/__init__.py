"""``modelopt.torch.opt`` save / restore for quantized models (reference opt/conversion.py:445-700).

Only the quantization mode exists in this build, so the modelopt state is the reference's layout
restricted to it::

    {"modelopt_state_dict": [("quantize", {"config": <QuantizeConfig dict>,
                                           "metadata": {"quantizer_state": {name: state}}})],
     "modelopt_version": "<version>"}

``restore_from_modelopt_state`` re-inserts the quantizers into an unquantized model of the same
architecture (module swap + ``quant_cfg``), promotes static-block quantizers, and sets every
quantizer's properties and buffer shapes, so that ``model.load_state_dict`` then loads the amax /
pre-quant-scale values (reference conversion.py:93-168).
"""

from __future__ import annotations

import os
from typing import Any, BinaryIO

import torch
import torch.nn as nn

__all__ = ["modelopt_state", "restore", "restore_from_modelopt_state", "save"]

MODELOPT_VERSION = "0.0.0+mi355x"
# plain builtins a quantizer state may hold (e.g. a ``slice`` for padded block views)
_SAFE_GLOBALS = [slice]


def modelopt_state(model: nn.Module) -> dict[str, Any]:
    """The modelopt state of ``model`` (reference conversion.py:445-492); no weights."""
    from ..quantization.conversion import quantizer_state

    entry = model.__dict__.get("_modelopt_amd_mode")
    if entry is None:
        return {"modelopt_state_dict": [], "modelopt_version": MODELOPT_VERSION}
    config = entry["config"]
    modes = [("quantize", {"config": config, "metadata": {"quantizer_state": quantizer_state(model)}})]
    if "compress" in entry:  # mtq.compress (reference compress.py:179-193)
        modes.append(("real_quantize", {"config": entry["compress"]["config"],
                                        "metadata": _compress_metadata(model)}))
    return {"modelopt_state_dict": modes, "modelopt_version": MODELOPT_VERSION}


def _compress_metadata(model: nn.Module) -> dict[str, Any]:
    from ..quantization.compress import RealQuantLinear
    from ..quantization.qtensor import QTensorWrapper

    meta: dict[str, Any] = {"real_quantizer_state": {}, "q_tensor_state": {}}
    for name, m in model.named_modules():
        # RealQuantLinear modules, and any other module whose weight was packed (an nn.Embedding
        # whose weight quantizer a config enabled is compressed by the reference too)
        packed = isinstance(m._parameters.get("weight"), QTensorWrapper)
        if isinstance(m, RealQuantLinear) or (packed and hasattr(m, "weight_quantizer")):
            meta["real_quantizer_state"][name] = m.weight_quantizer.get_modelopt_state()
            if packed:
                st = m.weight.get_state()
                md = dict(st["metadata"])
                md["qtensor_class"] = md["qtensor_class"].__name__  # a name, not a class object
                meta["q_tensor_state"][name] = {**st, "metadata": md}
    return meta


def _validate(state: Any) -> None:
    if not isinstance(state, dict):
        raise TypeError(f"Invalid modelopt state file: expected a dict, got {type(state).__name__}.")
    if "modelopt_state_dict" not in state or not isinstance(state["modelopt_state_dict"], list):
        raise ValueError("Invalid modelopt state: missing 'modelopt_state_dict' list.")
    for mode in state["modelopt_state_dict"]:
        if not (isinstance(mode, (tuple, list)) and len(mode) == 2 and isinstance(mode[1], dict)):
            raise ValueError(f"Invalid modelopt state entry {mode!r}.")
        if mode[0] not in ("quantize", "max", "mse", "awq_lite", "awq_clip", "awq_full", "real_quantize"):
            raise NotImplementedError(f"modelopt_amd: mode {mode[0]!r} is out of scope")


def restore_from_modelopt_state(
    model: nn.Module, modelopt_state: dict[str, Any] | None = None,
    modelopt_state_path: str | os.PathLike | None = None,
) -> nn.Module:
    """Re-apply the saved quantization to an unquantized model (reference conversion.py:577-647)."""
    from ..quantization.config import QuantizeConfig
    from ..quantization.conversion import replace_quant_module, restore_quantizer_state, set_quantizer_by_cfg
    from ..quantization.utils.names import is_quantized

    if modelopt_state is None:
        if modelopt_state_path is None:
            raise ValueError("Either modelopt_state or modelopt_state_path must be provided.")
        with torch.serialization.safe_globals(_SAFE_GLOBALS):
            modelopt_state = torch.load(modelopt_state_path, map_location="cpu", weights_only=True)
    _validate(modelopt_state)
    for mode, entry in modelopt_state["modelopt_state_dict"]:
        if mode == "real_quantize":
            _restore_compressed(model, entry)
            continue
        if mode != "quantize":
            continue  # calibration modes carry no architecture change
        config = QuantizeConfig(**entry["config"])
        if not is_quantized(model):
            replace_quant_module(model)
        set_quantizer_by_cfg(model, config.quant_cfg)
        restore_quantizer_state(model, config, entry["metadata"])
        model.__dict__["_modelopt_amd_mode"] = {"config": entry["config"]}
    return model


def _restore_compressed(model: nn.Module, entry: dict) -> None:
    """Re-create the packed weights' containers (shape / dtype / QTensor class) and the weight
    quantizers' scale buffers so ``load_state_dict`` fills them (reference compress.py:136-176)."""
    from ..quantization import qtensor as qt
    from ..quantization.compress import CompressConfig, compress_convert
    from ..quantization.qtensor import QTensorWrapper

    cfg = CompressConfig(entry["config"].get("compress"), entry["config"].get("quant_gemm", True))
    compress_convert(model, cfg, skip_real_quantize_weight=True)
    meta = entry["metadata"]
    for name, m in model.named_modules():
        if name in meta.get("real_quantizer_state", {}):
            m.weight_quantizer.set_from_modelopt_state(meta["real_quantizer_state"][name])
            m.weight_quantizer._dequantize = True
        if name in meta.get("q_tensor_state", {}):
            st = meta["q_tensor_state"][name]
            md = dict(st["metadata"])
            md["qtensor_class"] = getattr(qt, md["qtensor_class"])
            dev = m.weight.device
            m._parameters["weight"] = QTensorWrapper(
                torch.empty(st["quantized_data.shape"], dtype=st["quantized_data.dtype"], device=dev), metadata=md
            )
    model.__dict__.setdefault("_modelopt_amd_mode", {"config": {}})["compress"] = {"config": dict(cfg), "metadata": {}}


def save(model: nn.Module, f: str | os.PathLike | BinaryIO, **kwargs) -> None:
    """Model weights + modelopt state in one file (reference conversion.py:495-513)."""
    torch.save({"modelopt_state": modelopt_state(model), "model_state_dict": model.state_dict()}, f, **kwargs)


def restore(model: nn.Module, f: str | os.PathLike | BinaryIO, **kwargs) -> nn.Module:
    """Load a ``save`` checkpoint into ``model`` (reference conversion.py:650-700).  Loaded with
    ``weights_only=True``: the state holds only tensors, containers, numbers, strings, dtypes
    and sizes."""
    kwargs.setdefault("map_location", "cpu")
    kwargs.setdefault("weights_only", True)
    with torch.serialization.safe_globals(_SAFE_GLOBALS):
        objs = torch.load(f, **kwargs)
    model = restore_from_modelopt_state(model, objs["modelopt_state"])
    model.load_state_dict(objs["model_state_dict"])
    return model
