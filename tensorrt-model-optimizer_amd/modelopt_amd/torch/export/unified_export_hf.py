"""Unified Hugging Face checkpoint export (reference: export/unified_export_hf.py).

``export_hf_checkpoint(model, export_dir=...)`` turns a calibrated fake-quant model into the
deployable checkpoint the reference writes: packed low-precision weights (FP8 bytes, INT4 / NVFP4 /
MXFP4 nibble pairs) with ``weight_scale`` / ``weight_scale_2`` / ``input_scale`` /
``pre_quant_scale`` tensors under the original HF names, ``hf_quant_config.json`` and the
``quantization_config`` entry of ``config.json``.  Steps (reference :928-1023):

1. ``requantize_resmooth_fused_llm_layers`` -- a quantizer-free dummy forward finds linears fed by
   the same tensor (q/k/v, gate/up, experts) and unifies their pre-quant scales / amax, folding
   AWQ pre-quant scales into the preceding norm (:433-542);
2. per quantized module: scales + packed weight (HIP export kernels) (:569-810), fused MoE
   experts split into per-expert ``gate_proj`` / ``up_proj`` / ``down_proj`` (moe_utils.py:48);
3. quantizer state dropped / renamed (``postprocess_state_dict``), files written.
"""

from __future__ import annotations

import copy
import importlib
import json
import re
import warnings
from collections import defaultdict
from pathlib import Path

import torch
import torch.nn as nn

from ..quantization.conversion import set_quantizer_by_cfg_context
from ..quantization.nn import SequentialQuantizer, TensorQuantizer
from ..quantization.utils.names import is_quantized_linear, quantizer_attr_names
from .convert_hf_config import convert_hf_quant_config_format
from .quant_aware_conversion import (
    QuantConversionUnsupportedError,
    build_reverse_name_mapper,
    revert_quant_config_names,
    revert_weight_conversion_quant_aware,
)
from .model_config import (
    NVFP4_FAMILY,
    QUANTIZATION_FP8,
    QUANTIZATION_FP8_PB_REAL,
    QUANTIZATION_MXFP8,
    QUANTIZATION_NONE,
    QUANTIZATION_NVFP4_SVDQUANT,
    QUANTIZATION_W4A8_AWQ,
)
from .quant_utils import (
    _div,
    fuse_prequant_layernorm,
    fuse_prequant_to_linear,
    get_activation_scaling_factor,
    get_quant_config,
    get_quantization_format,
    get_weight_block_size,
    get_weight_scaling_factor,
    get_weight_scaling_factor_2,
    nvfp4_weights_scaling_factor,
    nvfp4_weights_scaling_factor_from_quantizer,
    postprocess_state_dict,
    preprocess_linear_fusion,
    to_quantized_weight,
)

__all__ = ["export_hf_checkpoint", "requantize_resmooth_fused_llm_layers"]


def _is_enabled(q) -> bool:
    if isinstance(q, SequentialQuantizer):
        return any(x.is_enabled for x in q)
    return isinstance(q, TensorQuantizer) and q.is_enabled


def _is_layernorm(module) -> bool:
    n = type(module).__name__.lower()
    return isinstance(module, nn.LayerNorm) or "rmsnorm" in n or "layernorm" in n


def collect_shared_input_modules(model, dummy_forward, collect_layernorms=False):
    """Linears that see the same input tensor, and which norm produced it (reference :280-348)."""
    input_to_linear = defaultdict(list)
    output_to_layernorm = defaultdict(lambda: None) if collect_layernorms else None
    handles = []

    def in_hook(module, inp, out):
        if len(inp) > 0 and isinstance(inp[0], torch.Tensor):
            input_to_linear[inp[0]].append(module)

    def out_hook(module, inp, out):
        if output_to_layernorm is not None and isinstance(out, torch.Tensor):
            output_to_layernorm[out] = module

    for name, module in model.named_modules():
        if collect_layernorms and _is_layernorm(module):
            module.name = name
            handles.append(module.register_forward_hook(out_hook))
        elif is_quantized_linear(module) and (
            _is_enabled(module.input_quantizer) or _is_enabled(module.weight_quantizer)
        ):
            module.name = name
            handles.append(module.register_forward_hook(in_hook))
    if not handles:
        return input_to_linear, output_to_layernorm
    use_cache = getattr(getattr(model, "config", None), "use_cache", None)
    try:
        if use_cache is not None:
            model.config.use_cache = False
        with torch.no_grad(), set_quantizer_by_cfg_context(model, [{"quantizer_name": "*", "enable": False}]):
            dummy_forward()
    finally:
        if use_cache is not None:
            model.config.use_cache = use_cache
        for h in handles:
            h.remove()
    return input_to_linear, output_to_layernorm


def requantize_resmooth_fused_llm_layers(model: nn.Module):
    """reference :433-542 (LLM path)."""
    fmt = get_quantization_format(model)
    if fmt is not None and "nvfp4_awq" in fmt.lower():
        fuse_prequant_to_linear(model)
    module_names = {n for n, _ in model.named_modules()}
    device = next(model.parameters()).device

    def dummy():
        model(torch.ones([1, 2], dtype=torch.long, device=device))

    input_to_linear, output_to_layernorm = collect_shared_input_modules(model, dummy, collect_layernorms=True)
    fused = {}
    for tensor, modules in input_to_linear.items():
        gfmt = get_quantization_format(modules[0]) if modules else fmt
        if len(modules) > 1 and gfmt not in (QUANTIZATION_FP8, QUANTIZATION_NONE, QUANTIZATION_FP8_PB_REAL):
            preprocess_linear_fusion(modules)
            fused[modules[0].name] = [m.name for m in modules]
        if (
            output_to_layernorm is not None and gfmt is not None and gfmt != QUANTIZATION_NONE
            and "awq" in gfmt and tensor in output_to_layernorm and output_to_layernorm[tensor] is not None
        ):
            fuse_prequant_layernorm(output_to_layernorm[tensor], modules)
    # experts the dummy forward did not reach (iterable experts named experts.N)
    for name, names in fused.items():
        if re.search(r"experts?\.\d+", name):
            e = 0
            while True:
                new = re.sub(r"(experts?\.)\d+", rf"\g<1>{e}", name, count=1)
                if new in fused:
                    e += 1
                    continue
                if new not in module_names:
                    break
                mods = [model.get_submodule(re.sub(r"(experts?\.)\d+", rf"\g<1>{e}", n)) for n in names]
                preprocess_linear_fusion(mods)
                e += 1


def _export_quantized_weight(sub_module: nn.Module, dtype: torch.dtype, weight_name: str = "weight"):
    """Scales + packed weight for one weight attribute (reference :569-810)."""
    fmt = get_quantization_format(sub_module)
    if fmt == QUANTIZATION_NONE:
        return
    block_size = get_weight_block_size(sub_module, weight_name)
    names = quantizer_attr_names(weight_name)
    weight = getattr(sub_module, weight_name)
    wq = getattr(sub_module, names.weight_quantizer)
    iq = getattr(sub_module, names.input_quantizer, None)
    oq = getattr(sub_module, names.output_quantizer, None)

    if fmt == QUANTIZATION_FP8:
        wq._amax = wq._amax.to(torch.float32)
        if wq._amax.dim() == 1:
            wsf = torch.tensor(wq.amax.item() / wq.maxbound)
        else:
            wsf = _div(wq.amax, wq.maxbound).clone().detach()
        sub_module.register_buffer(names.weight_scale, wsf)
        if hasattr(iq, "_amax"):
            iq._amax = iq._amax.to(torch.float32)
            sub_module.register_buffer(names.input_scale, get_activation_scaling_factor(sub_module, names.input_quantizer).squeeze())
        if hasattr(oq, "_amax"):
            oq._amax = oq._amax.to(torch.float32)
    else:
        if fmt == QUANTIZATION_MXFP8:
            # E8M0 bytes per 32 (reference unified_export_hf.py:671-680)
            from ..quantization.qtensor import MXFP8QTensor

            sub_module.register_buffer(
                names.weight_scale, MXFP8QTensor.get_weights_scaling_factor_from_quantizer(weight, wq)
            )
            if getattr(wq, "_scale", None) is not None:
                del wq._scale
        else:
            sub_module.register_buffer(names.weight_scale, get_weight_scaling_factor(sub_module, weight_name))
        if iq is not None and iq.is_enabled and iq.amax is not None:
            sub_module.register_buffer(names.input_scale, get_activation_scaling_factor(sub_module, names.input_quantizer).squeeze())

    if fmt in (*NVFP4_FAMILY, QUANTIZATION_W4A8_AWQ) and fmt != QUANTIZATION_NVFP4_SVDQUANT:
        sub_module.register_buffer(names.weight_scale_2, get_weight_scaling_factor_2(sub_module, weight_name).squeeze())

    weight_scale = getattr(sub_module, names.weight_scale, None)
    weight_scale_2 = getattr(sub_module, names.weight_scale_2, None)
    if fmt in NVFP4_FAMILY and fmt not in ("w4a8_nvfp4_fp8",):
        from ..quantization.nn.modules.tensor_quantizer import StaticBlockScaleQuantizer

        if isinstance(wq, StaticBlockScaleQuantizer) and wq.global_amax is not None:
            weight_scale = nvfp4_weights_scaling_factor_from_quantizer(wq, weight, weight_scale_2)
        else:
            weight_scale = nvfp4_weights_scaling_factor(weight, block_size, weight_scale_2)
    qweight = to_quantized_weight(weight.to(dtype), weight_scale, fmt, weight_scale_2, block_size)
    setattr(sub_module, weight_name, nn.Parameter(qweight, requires_grad=False))
    if weight_scale is not None:
        sub_module.register_buffer(names.weight_scale, weight_scale)


def _export_fused_experts(module: nn.Module, dtype: torch.dtype):
    """Split fused [E, 2I, H] / [E, H, I] expert weights into per-expert gate/up/down projections
    with their own scales (reference moe_utils.py:48-200)."""
    n = module.num_experts
    first_attr = getattr(module, "_first_proj_attr", "gate_up_proj")
    first_iq = getattr(module, f"{first_attr}_input_quantizer")
    first_wqs = getattr(module, f"{first_attr}_weight_quantizers")
    down_iq = module.down_proj_input_quantizer
    first = getattr(module, first_attr).data
    down = module.down_proj.data
    inter = first.shape[1] // 2
    for idx in range(n):
        fq = first_wqs[idx]
        if getattr(fq, "is_enabled", False) and (not hasattr(fq, "_amax") or fq._amax is None or torch.all(fq._amax == 0)):
            fq.amax = first[idx].abs().amax().to(torch.float32)
            warnings.warn(f"Expert {idx} gate_up_proj weight quantizer was not calibrated; using the fused-tensor amax.")
        expert = nn.Module()
        for proj, w, start, total, uses_first in (
            ("gate_proj", first[idx, :inter, :], 0, first.shape[1], True),
            ("up_proj", first[idx, inter:, :], inter, first.shape[1], True),
            ("down_proj", down[idx], 0, down.shape[1], False),
        ):
            src = first_wqs[idx] if uses_first else module.down_proj_weight_quantizers[idx]
            wq = copy.deepcopy(src) if uses_first else src
            a = getattr(wq, "_amax", None)
            if a is not None and a.dim() >= 1 and a.numel() > 1 and a.shape[0] == total:
                wq._amax = a[start : start + w.shape[0]].contiguous()
            if getattr(wq, "is_enabled", False) and (getattr(wq, "_amax", None) is None or torch.all(wq._amax == 0)):
                wq.amax = w.abs().amax().to(torch.float32)
            holder = _ExpertLinear(nn.Parameter(w.contiguous(), requires_grad=False), wq,
                                   first_iq if uses_first else down_iq)
            _export_quantized_weight(holder, dtype)
            out = nn.Module()
            out.weight = holder.weight
            for key in ("weight_scale", "weight_scale_2", "input_scale"):
                if key in holder._buffers:
                    out.register_buffer(key, holder._buffers[key])
            expert.add_module(proj, out)
        module.add_module(str(idx), expert)
    for attr in (first_attr, "down_proj"):
        delattr(module, attr)
    for attr in (f"{first_attr}_weight_quantizers", "down_proj_weight_quantizers",
                 f"{first_attr}_input_quantizer", "down_proj_input_quantizer"):
        if hasattr(module, attr):
            delattr(module, attr)


class _ExpertLinear(nn.Module):
    """A per-expert projection view with the quantizer attributes export reads."""

    def __init__(self, weight, weight_quantizer, input_quantizer):
        super().__init__()
        self.weight = weight
        self.weight_quantizer = weight_quantizer
        self.input_quantizer = copy.deepcopy(input_quantizer)


def _process_quantized_modules(model: nn.Module, dtype: torch.dtype):
    for name, m in list(model.named_modules()):
        if hasattr(m, "gate_up_proj_weight_quantizers") or hasattr(m, "up_proj_weight_quantizers"):
            _export_fused_experts(m, dtype)
        elif is_quantized_linear(m):
            if get_quantization_format(m) == QUANTIZATION_NONE:
                continue
            try:
                _export_quantized_weight(m, dtype)
            except AssertionError as e:
                raise AssertionError(f"Failed to export module '{name}' (type={type(m).__name__}): {e}") from e
        elif isinstance(m, nn.Embedding) and hasattr(m, "weight_quantizer"):
            # a quantized embedding table, unless its weight is tied (reference
            # hf_export_handlers.py:154-182)
            if get_quantization_format(m) == QUANTIZATION_NONE:
                continue
            tied = [n for n, o in model.named_modules() if o is not m and getattr(o, "weight", None) is m.weight]
            if tied:
                warnings.warn(f"Skipping quantized weight packing for embedding '{name}': its weight is shared with {tied}.")
                continue
            _export_quantized_weight(m, dtype)


def _export_dtype(model, dtype):
    cfg_dtype = getattr(model.config, "torch_dtype", None) or getattr(model.config, "dtype", None)
    if isinstance(cfg_dtype, str):
        cfg_dtype = getattr(torch, cfg_dtype)
    if dtype is None:
        return cfg_dtype or next(model.parameters()).dtype
    if cfg_dtype is not None and dtype != cfg_dtype:
        warnings.warn(f"Model's original dtype ({cfg_dtype}) differs from target dtype ({dtype}).")
    return dtype


def _export_transformers_checkpoint(model: nn.Module, dtype=None):
    dtype = _export_dtype(model, dtype)
    requantize_resmooth_fused_llm_layers(model)
    quant_config = get_quant_config(model)
    _process_quantized_modules(model, dtype)
    state = postprocess_state_dict(model.state_dict(), 448, quant_config["quantization"]["kv_cache_quant_algo"])
    return state, quant_config


def export_hf_checkpoint(model, dtype: torch.dtype | None = None, export_dir="/tmp/modelopt_amd_export",
                         save_modelopt_state: bool = False, extra_state_dict: dict | None = None,
                         max_shard_size="10GB", **kwargs):
    """Write the packed checkpoint + configs to ``export_dir`` (reference :1491-1646)."""
    export_dir = Path(export_dir)
    export_dir.mkdir(parents=True, exist_ok=True)
    post_state, hf_quant_config = _export_transformers_checkpoint(model, dtype)
    state = {**post_state, **(extra_state_dict or {})}
    # back to the hub checkpoint's names (transformers-5 load-time conversions), scales attached
    try:
        mapper = build_reverse_name_mapper(model)
        state = revert_weight_conversion_quant_aware(model, state)
        if mapper is not None:
            revert_quant_config_names(hf_quant_config.get("quantization", {}), mapper)
    except QuantConversionUnsupportedError as exc:
        warnings.warn(f"Quant-aware reverse weight conversion skipped ({exc}); in-memory names kept.")
    gc = getattr(model, "generation_config", None)
    if gc is not None and (getattr(gc, "top_k", None) is not None or getattr(gc, "top_p", None) is not None):
        gc.do_sample = True
    # transformers' own revert (which chokes on 0-d scales) must not run on the reverted dict
    patches = []
    for mod_path in ("transformers.core_model_loading", "transformers.modeling_utils"):
        try:
            mod = importlib.import_module(mod_path)
        except ImportError:
            continue
        if hasattr(mod, "revert_weight_conversion"):
            patches.append((mod, mod.revert_weight_conversion))
            mod.revert_weight_conversion = lambda model, state_dict: state_dict
    try:
        model.save_pretrained(export_dir, state_dict=state, max_shard_size=max_shard_size)
    finally:
        for mod, orig in patches:
            mod.revert_weight_conversion = orig
    q = hf_quant_config.get("quantization", {})
    quantization_config = None
    if q.get("quant_algo") is not None or q.get("kv_cache_quant_algo") is not None:
        with open(export_dir / "hf_quant_config.json", "w") as f:
            json.dump(hf_quant_config, f, indent=4)
        quantization_config = convert_hf_quant_config_format(hf_quant_config)
    cfg_path = export_dir / "config.json"
    cfg = json.loads(cfg_path.read_text())
    if quantization_config is not None:
        cfg["quantization_config"] = quantization_config
    cfg_path.write_text(json.dumps(cfg, indent=4))
