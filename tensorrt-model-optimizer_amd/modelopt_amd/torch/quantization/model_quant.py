"""User-facing PTQ API: ``mtq.quantize`` / ``mtq.calibrate`` (reference: model_quant.py).

``quantize(model, config, forward_loop)`` = convert (insert quantizers, apply the ordered
wildcard ``quant_cfg``) + ``calibrate(model, config["algorithm"], forward_loop)``, as in
model_quant.py:147-250.  The reference routes both through its mode framework (apply_mode /
QuantizeModeDescriptor, mode.py); here they are direct calls with the same effects, the config is
recorded on ``model._modelopt_amd_mode`` and ``mto.modelopt_state`` reads the quantizer state off
the model when it is saved.
"""

from __future__ import annotations

import contextlib
import fnmatch
import inspect
import warnings
from collections.abc import Callable
from typing import Any

import torch
import torch.nn as nn

from .config import QuantizeConfig, algorithm_config
from .conversion import set_quantizer_attributes_partial
from .layerwise import layerwise_calibrate
from .model_calib import awq, max_calibrate, mse_calibrate
from .nn.modules.quant_module import QuantModule
from .nn.modules.tensor_quantizer import SequentialQuantizer, TensorQuantizer
from .utils.core_utils import gc_paused as _gc_paused
from .utils.names import is_quantized

__all__ = [
    "calibrate",
    "compute_quantization_mse",
    "temporarily_fold_weights",
    "disable_quantizer",
    "enable_quantizer",
    "fold_weight",
    "postprocess_amax",
    "print_quant_summary",
    "quantize",
]


def _apply_algorithm(model, algo_cfg, forward_loop):
    if algo_cfg is None:
        return
    kwargs = algo_cfg.model_dump()
    method = kwargs.pop("method")
    ratio = kwargs.pop("moe_calib_experts_ratio", None)
    if ratio is not None:
        # reference mode.py:240-247: set on every sparse sequential MoE block; transformers-5
        # fused-expert blocks have no such wrapper there either, so the ratio has no effect on them
        assert isinstance(ratio, (int, float)) and 0 < ratio <= 1, f"Invalid moe_calib_experts_ratio {ratio!r}"
        for module in model.modules():
            if hasattr(module, "_moe_calib_experts_ratio"):
                module._moe_calib_experts_ratio = ratio
    layerwise = kwargs.pop("layerwise", None) or {}
    if layerwise is True:
        layerwise = {"enable": True}
    if method == "max":
        kwargs.pop("shared_states", None)
        func = max_calibrate
    elif method == "mse":
        func = mse_calibrate
    elif method in ("awq_lite", "awq_full", "awq_clip"):
        kwargs["algorithm"] = method
        func = awq
    elif method is None:
        return
    else:
        raise NotImplementedError(f"calibration algorithm {method!r}")
    if layerwise.get("enable", False):
        # reference mode.py:250-272
        if layerwise.get("checkpoint_dir") and not layerwise.get("enable"):
            raise ValueError("layerwise.checkpoint_dir requires layerwise.enable=True")
        if forward_loop is None:
            raise ValueError("forward_loop is required for calibration but got None.")
        layerwise_calibrate(
            model, forward_loop, func,
            checkpoint_dir=layerwise.get("checkpoint_dir"),
            get_qdq_activations_from_prev_layer=layerwise.get("get_qdq_activations_from_prev_layer", False),
            save_every=layerwise.get("save_every", 1),
            calib_mutates_weights=layerwise.get("calib_mutates_weights", True),
            **kwargs,
        )
    else:
        func(model, forward_loop, **kwargs)


def _validate_quantizer_attrs(model: nn.Module) -> None:
    """``validate_attr`` of every quantizer's ``_amax`` / ``_pre_quant_scale`` (reference :121-127)
    as one batched check per device -- each per-quantizer check is three host syncs, ~1.3 k for
    Llama-3-8B.  Only when the batch holds a negative / inf / NaN value are the quantizers
    checked one by one, which emits the reference's per-quantizer warnings."""
    from .calib.max import _bad_flags

    found = []
    for name, module in model.named_modules():
        if isinstance(module, TensorQuantizer):
            for attr_name in ["_amax", "_pre_quant_scale"]:
                v = getattr(module, attr_name, None)
                if isinstance(v, torch.Tensor) and not v.is_meta:
                    found.append((name, module, attr_name, v))
    groups: dict = {}
    for item in found:
        groups.setdefault((item[3].device, item[3].dtype), []).append(item)
    by_dev: dict = {}
    for (dev, dt), items in groups.items():
        flat = torch.cat([v.detach().reshape(-1) for *_, v in items])
        if dt in (torch.float32, torch.bfloat16, torch.float16):
            flags = _bad_flags(flat)  # NaN, inf, negative: the library's kernel on the GPU
        else:
            flags = torch.stack([((flat < 0) | ~torch.isfinite(flat)).any()] * 3).to(torch.int32)
        by_dev.setdefault(dev, []).append((flags, items))
    for checks in by_dev.values():
        bad = torch.cat([c for c, _ in checks]).tolist()  # one host sync per device
        for i, (_, items) in enumerate(checks):
            if any(bad[3 * i : 3 * i + 3]):
                for name, module, attr_name, _ in items:
                    module.validate_attr(attr_name=attr_name, warn_error=True, name=name)


def calibrate(model: nn.Module, algorithm="max", forward_loop: Callable | None = None) -> nn.Module:
    """Calibrate the quantizers of ``model`` (reference :64-129)."""
    if forward_loop is not None:
        nargs = len(inspect.signature(forward_loop).parameters)
        if nargs == 0:
            warnings.warn(
                "forward_loop should take model as argument, but got forward_loop without any arguments.",
                DeprecationWarning,
            )
            original = forward_loop

            def forward_loop(model):  # noqa: F811
                return original()

    is_training = model.training
    model.eval()
    _apply_algorithm(model, algorithm_config(algorithm), forward_loop)
    with _gc_paused():
        _validate_quantizer_attrs(model)
        model.train(is_training)
    return model


def quantize(model: nn.Module, config: dict[str, Any] | QuantizeConfig, forward_loop: Callable | None = None) -> nn.Module:
    """Quantize and calibrate ``model`` in place (reference :147-250)."""
    if isinstance(config, dict):
        config = QuantizeConfig(**config)
    from .conversion import replace_quant_module, set_quantizer_by_cfg

    model.__dict__["_modelopt_amd_mode"] = {"config": config.model_dump()}  # for mto.modelopt_state
    with _gc_paused():
        if not is_quantized(model):
            # convert_to_quantized_model minus its metadata dict: calibrate() records the state once
            replace_quant_module(model)
        set_quantizer_by_cfg(model, config.quant_cfg)
    return calibrate(model, config.algorithm, forward_loop)




def postprocess_amax(model: nn.Module, key: str, post_process_fn) -> nn.Module:
    """Apply ``post_process_fn`` to the amax of quantizers matching ``key`` (reference :132-145)."""
    for name, module in model.named_modules():
        if not isinstance(module, TensorQuantizer) or not fnmatch.fnmatch(name, key):
            continue
        if module.amax is not None:
            module.amax = post_process_fn(module.amax)
    return model


def disable_quantizer(model: nn.Module, wildcard_or_filter_func: str | Callable):
    set_quantizer_attributes_partial(model, wildcard_or_filter_func, {"enable": False})


def enable_quantizer(model: nn.Module, wildcard_or_filter_func: str | Callable):
    set_quantizer_attributes_partial(model, wildcard_or_filter_func, {"enable": True})


def print_quant_summary(model: nn.Module, output_dir: str | None = None):
    lines = []
    for name, mod in model.named_modules():
        if isinstance(mod, (TensorQuantizer, SequentialQuantizer)):
            lines.append(f"{name:80} {mod}")
    lines.append(f"{len(lines)} TensorQuantizers found in model")
    text = "\n".join(lines)
    if output_dir:
        import os

        os.makedirs(output_dir, exist_ok=True)
        with open(os.path.join(output_dir, ".quant_summary.txt"), "w") as f:
            f.write(text)
    else:
        print(text)


@torch.no_grad()
def fold_weight(model: nn.Module, keep_attrs: bool = False):
    """Bake the weight fake-quant into the weights (reference :728-738)."""
    for _, module in model.named_modules():
        if isinstance(module, QuantModule):
            module.fold_weight(keep_attrs)


@contextlib.contextmanager
def temporarily_fold_weights(model: nn.Module, snapshot_device: torch.device | str | None = None):
    """Fold the fake-quant weights for a frozen inference region, restoring them on exit
    (reference model_quant.py:740-806): each QuantModule's ``fold_weight(keep_attrs=True)``, the
    quantizers' properties restored by ``preserve_quantizer_attributes_context``, and every
    weight a quantization / pre_quant_scale / rotation changes copied back in place from a
    snapshot (on ``snapshot_device``, default the weight's own), exceptions included.
    SequentialQuantizer weights are not supported (NotImplementedError), as in the reference."""
    from .conversion import preserve_quantizer_attributes_context

    pairs = []
    for module in model.modules():
        if not isinstance(module, QuantModule):
            continue
        for weight, q in module.iter_weights_for_calibration():
            if not isinstance(weight, torch.Tensor):
                continue
            if isinstance(q, SequentialQuantizer):
                raise NotImplementedError("temporarily_fold_weights does not support SequentialQuantizer")
            if not isinstance(q, TensorQuantizer) or not q.fake_quant:
                continue
            pairs.append((weight.to_local() if hasattr(weight, "to_local") else weight, q))
    snapshots = {}
    for w, q in pairs:
        if q.is_enabled or q.pre_quant_scale is not None or q.rotate_is_enabled:
            if id(w) not in snapshots:
                snapshots[id(w)] = (w, w.detach().clone() if snapshot_device is None
                                    else w.detach().to(snapshot_device, copy=True))
    with preserve_quantizer_attributes_context(model):
        try:
            fold_weight(model, keep_attrs=True)
            yield
        finally:
            with torch.no_grad():
                for w, snap in snapshots.values():
                    w.copy_(snap)


@torch.no_grad()
def compute_quantization_mse(model: nn.Module, forward_loop, wildcards="*") -> dict[str, float]:
    """Mean over the ``forward_loop`` batches of mean((x - qdq(x))^2) for every enabled fake-quant
    TensorQuantizer whose name matches ``wildcards`` (fnmatch patterns or callables; reference
    model_quant.py:809-882); disabled / non-fake quantizers are absent from the result."""
    pats = wildcards if isinstance(wildcards, list) else [wildcards]

    def match(name):
        return any(fnmatch.fnmatch(name, w) if isinstance(w, str) else w(name) for w in pats)

    acc: dict[str, list] = {}
    hooks = []
    for name, m in model.named_modules():
        if not isinstance(m, TensorQuantizer) or not match(name):
            continue
        if not (m._if_quant and m._fake_quant) or m._disabled:
            continue
        acc[name] = [0.0, 0]

        def hook(mod, inp, out, a=acc[name]):
            a[0] += torch.mean((inp[0].detach().float() - out.detach().float()) ** 2).item()
            a[1] += 1

        hooks.append(m.register_forward_hook(hook))
    try:
        forward_loop(model)
    finally:
        for h in hooks:
            h.remove()
    return {n: s / c for n, (s, c) in acc.items() if c > 0}

