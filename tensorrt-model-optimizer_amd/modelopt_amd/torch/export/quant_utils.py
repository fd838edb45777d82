"""Quantized-checkpoint helpers: format detection, scaling factors, weight packing, config.

Reference: modelopt/torch/export/quant_utils.py (format detection :485-603, scaling factors
:225-362, packing :792-938, fusion preprocessing :1285-1547, config :606-790 / :1583-1705,
state-dict postprocessing :980-1110) and qtensor/{nvfp4,mxfp4}_tensor.py.  The byte work (FP8
casts, INT4 / NVFP4 / MXFP4 packing) runs in the HIP export kernels (`mtq_export_*`); the scale
math is a handful of small device ops written as the reference's torch expressions so the
values are bit-identical.
"""

from __future__ import annotations

import warnings
from typing import Any

import torch
import torch.nn as nn

from modelopt_amd._ext import ops as _ops

from ..quantization.model_calib import enable_stats_collection, finish_stats_collection
from ..quantization.nn import SequentialQuantizer, TensorQuantizer
from ..quantization.nn.modules.quant_module import QuantModule
from ..quantization.nn.modules.tensor_quantizer import StaticBlockScaleQuantizer
from ..quantization.utils.names import quantizer_attr_names, representative_weight_quantizer, weight_attr_names
from .model_config import (
    KV_CACHE_FP8,
    KV_CACHE_NVFP4,
    KV_CACHE_NVFP4_AFFINE,
    NVFP4_FAMILY,
    QUANTIZATION_FP8,
    QUANTIZATION_FP8_PB_REAL,
    QUANTIZATION_FP8_PB_WO,
    QUANTIZATION_FP8_PC_PT,
    QUANTIZATION_INT4_AWQ,
    QUANTIZATION_INT8_SQ,
    QUANTIZATION_INT8_WO,
    QUANTIZATION_MXFP4,
    QUANTIZATION_MXFP8,
    QUANTIZATION_NONE,
    QUANTIZATION_NVFP4,
    QUANTIZATION_NVFP4_AWQ,
    QUANTIZATION_NVFP4_SVDQUANT,
    QUANTIZATION_W4A8_AWQ,
    QUANTIZATION_W4A8_MXFP4_FP8,
    QUANTIZATION_W4A8_NVFP4_FP8,
    QUANTIZATION_W4A16_NVFP4,
)

E2M1_MAX = 6.0
E4M3_MAX = 448.0


def _div(t: torch.Tensor, c) -> torch.Tensor:
    """IEEE fp32 ``t / c``.  torch on ROCm turns a division by a host scalar into a multiply by
    its reciprocal (1-ulp off the reference's CPU export); a device-tensor divisor is a true
    division."""
    t = t.float()
    if not isinstance(c, torch.Tensor):
        c = torch.tensor(float(c), dtype=torch.float32, device=t.device)
    return torch.div(t, c.to(device=t.device, dtype=torch.float32))


def _mean0(ts: list[torch.Tensor]) -> torch.Tensor:
    """torch.mean(torch.stack(ts), 0) as the CPU computes it for a few rows: a sequential fp32
    sum, then one true division."""
    acc = ts[0].float()
    for t in ts[1:]:
        acc = acc + t.float()
    return _div(acc, len(ts)).to(ts[0].dtype)


def _fp8_max_for_normalization(quantizer) -> float:
    bs = getattr(quantizer, "block_sizes", None) or {}
    return 256.0 if bool(bs.get("four_over_six", False)) else E4M3_MAX


# ---- format detection -------------------------------------------------------------------------
def _layer_format(layer: nn.Module, weight_name: str) -> str | None:
    """reference quant_utils.py:491-591 for one weight attribute."""
    names = quantizer_attr_names(weight_name)
    wq = representative_weight_quantizer(layer, weight_name)
    iq = getattr(layer, names.input_quantizer, None)
    if wq is None or not wq.is_enabled:
        return QUANTIZATION_NONE
    if isinstance(wq, SequentialQuantizer):
        assert len(wq) == 2 and wq[0].num_bits == 4 and wq[1].num_bits == (4, 3), (
            "Unsupported SequentialQuantizer configuration"
        )
        assert wq[0].block_sizes and wq[0].block_sizes[-1] > 0, "Invalid block_sizes for SequentialQuantizer"
        return QUANTIZATION_W4A8_AWQ
    if wq.num_bits == 4:
        assert wq.block_sizes and wq.block_sizes[-1] > 0, "Invalid block_sizes for INT4 quantizer"
        return QUANTIZATION_INT4_AWQ
    if wq.num_bits == 8:
        return QUANTIZATION_INT8_SQ if (iq is not None and iq.is_enabled) else QUANTIZATION_INT8_WO
    if wq.num_bits == (4, 3):
        if wq.block_sizes:
            assert wq.block_sizes[-1] > 0, "Invalid block_sizes for FP8 quantizer"
            bs = wq.block_sizes
            if isinstance(bs, dict) and bs.get("type", "static") == "dynamic" and bs.get("scale_bits") == (8, 0):
                return QUANTIZATION_MXFP8
            return QUANTIZATION_FP8_PB_WO if wq.fake_quant else QUANTIZATION_FP8_PB_REAL
        if wq.axis == 0:
            return QUANTIZATION_FP8_PC_PT
        return QUANTIZATION_FP8
    if wq.num_bits == (2, 1):
        bs = wq.block_sizes
        scale_bits = bs.get("scale_bits")
        if iq is not None and hasattr(wq, "svdquant_lora_a"):
            return QUANTIZATION_NVFP4_SVDQUANT
        if iq is not None and hasattr(iq, "_pre_quant_scale"):
            return QUANTIZATION_NVFP4_AWQ
        if getattr(layer, "fused_with_prequant", False):
            return QUANTIZATION_NVFP4_AWQ
        if (iq is None or not iq.is_enabled) and scale_bits == (4, 3):
            return QUANTIZATION_W4A16_NVFP4
        assert iq is not None, f"input_quantizer is None for {names}"
        fp8_in = iq.is_enabled and iq.num_bits == (4, 3) and iq.block_sizes is None
        if bs.get("type", "static") == "dynamic" and scale_bits == (8, 0) and fp8_in:
            return QUANTIZATION_W4A8_MXFP4_FP8
        if bs.get("type", "static") == "dynamic" and scale_bits == (4, 3) and fp8_in:
            return QUANTIZATION_W4A8_NVFP4_FP8
        if scale_bits == (4, 3):
            return QUANTIZATION_NVFP4
        if scale_bits == (8, 0):
            return QUANTIZATION_MXFP4
    raise NotImplementedError(f"Unsupported quantizer with num_bits: {wq.num_bits}")


def get_quantization_format(module) -> str | None:
    """First non-None format of the module's weights, then of its children (reference :485-603)."""
    for weight_name in weight_attr_names(module):
        fmt = _layer_format(module, weight_name)
        if fmt != QUANTIZATION_NONE:
            return fmt
    for _, layer in module.named_children():
        fmt = get_quantization_format(layer)
        if fmt != QUANTIZATION_NONE:
            return fmt
    return QUANTIZATION_NONE


def get_weight_block_size(module: nn.Module, weight_name: str = "weight") -> int:
    wq = representative_weight_quantizer(module, weight_name)
    if wq is None:
        return 0
    if isinstance(wq, SequentialQuantizer):
        wq = wq[0]
    if not wq.is_enabled:
        return 0
    return wq.block_sizes[-1] if wq.block_sizes else 0


# ---- NVFP4 scale helpers (qtensor/nvfp4_tensor.py) ----------------------------------------------
def _static_global_amax(wq):
    return getattr(wq, "global_amax", None) if isinstance(wq, StaticBlockScaleQuantizer) else None


def nvfp4_weights_scaling_factor_2_from_quantizer(wq) -> torch.Tensor:
    m = _fp8_max_for_normalization(wq)
    g = _static_global_amax(wq)
    if g is not None:
        return _div(g, E2M1_MAX * m)
    assert hasattr(wq, "_amax"), "Weight quantizer does not have attribute amax"
    return _div(wq._amax, E2M1_MAX * m)


def _cast_per_block_scale_to_fp8(scale, scale_max=None, fp8_max=E4M3_MAX):
    if scale_max is not None:
        scale = _div(scale.float() * fp8_max, scale_max)
    return scale.clamp(min=2**-9, max=E4M3_MAX).to(torch.float8_e4m3fn)


def nvfp4_weights_scaling_factor(weight, block_size, scale_2, keep_high_precision=False):
    """Dynamic per-block scale from the weight (nvfp4_tensor.py:169-203)."""
    assert block_size != 0 and weight.shape[-1] % block_size == 0, (
        "Weight shape is not divisible for block size for block quantization."
    )
    per_block_amax = weight.reshape(*weight.shape[:-1], -1, block_size).abs().amax(dim=-1).float()
    per_block_scale = _div(per_block_amax, E2M1_MAX * scale_2.to(per_block_amax.device).float())
    per_block_scale[per_block_scale == 0] = 1.0
    if not keep_high_precision:
        per_block_scale = _cast_per_block_scale_to_fp8(per_block_scale)
    return per_block_scale


def nvfp4_weights_scaling_factor_from_quantizer(wq, weight, scale_2=None, keep_high_precision=False):
    """Static (pre-computed per-block amax) or dynamic per-block scale (nvfp4_tensor.py:111-167)."""
    block_size = wq.block_sizes[-1]
    if scale_2 is None:
        scale_2 = nvfp4_weights_scaling_factor_2_from_quantizer(wq)
    g = _static_global_amax(wq)
    if g is not None:
        per_block_scale_max = _div(g, E2M1_MAX)
        per_block_scale = _div(wq._amax, E2M1_MAX)
        per_block_scale[per_block_scale == 0] = 1.0
        per_block_scale = per_block_scale.view(*weight.shape[:-1], weight.shape[-1] // block_size)
        if not keep_high_precision:
            per_block_scale = _cast_per_block_scale_to_fp8(
                per_block_scale, per_block_scale_max, _fp8_max_for_normalization(wq)
            )
        return per_block_scale
    return nvfp4_weights_scaling_factor(weight, block_size, scale_2, keep_high_precision)


# ---- scaling factors ----------------------------------------------------------------------------
def get_scaling_factor(quantizer: TensorQuantizer) -> torch.Tensor | None:
    """amax / maxbound (NVFP4: the global scale) (reference :225-242)."""
    if not quantizer.is_enabled:
        return None
    amax = quantizer.export_amax()
    if amax is None:
        return None
    if quantizer.num_bits == (2, 1):
        sf = nvfp4_weights_scaling_factor_2_from_quantizer(quantizer)
    else:
        sf = _div(amax, quantizer.maxbound)
    assert torch.all(sf > 0), f"scaling factor {sf} not positive."
    return sf


def get_activation_scaling_factor(module, input_quantizer_name="input_quantizer"):
    iq = getattr(module, input_quantizer_name, None)
    if iq is None:
        return None
    if get_quantization_format(module) in (QUANTIZATION_NVFP4, QUANTIZATION_NVFP4_AWQ, QUANTIZATION_NVFP4_SVDQUANT):
        if not iq.is_enabled:
            return None
        amax = iq.export_amax()
        if amax is None:
            return None
        sf = _div(amax, iq.maxbound * E4M3_MAX)
        assert torch.all(sf > 0), f" activation scaling factor {sf} not positive."
        return sf
    return get_scaling_factor(iq)


def get_weight_scaling_factor(module, weight_name="weight"):
    weight = getattr(module, weight_name)
    wq = getattr(module, quantizer_attr_names(weight_name).weight_quantizer, None)
    if wq is None:
        return None
    if isinstance(wq, SequentialQuantizer):
        return get_scaling_factor(wq[0])
    fmt = get_quantization_format(module)
    if fmt in NVFP4_FAMILY:
        if fmt == QUANTIZATION_W4A8_NVFP4_FP8:
            s2 = _div(wq._amax, 448.0)
        else:
            s2 = nvfp4_weights_scaling_factor_2_from_quantizer(wq)
        return nvfp4_weights_scaling_factor_from_quantizer(wq, weight, s2.to(weight.device))
    if fmt in (QUANTIZATION_W4A8_MXFP4_FP8, QUANTIZATION_MXFP4):
        _, sc = mxfp4_quantize(weight, wq.block_sizes[-1])
        return sc.reshape(*weight.shape[:-1], -1)
    return get_scaling_factor(wq)


def get_weight_scaling_factor_2(module, weight_name="weight"):
    wq = getattr(module, quantizer_attr_names(weight_name).weight_quantizer, None)
    if wq is None:
        return None
    fmt = get_quantization_format(module)
    if fmt in NVFP4_FAMILY:
        if fmt == QUANTIZATION_W4A8_NVFP4_FP8:
            return _div(wq._amax, 448.0)
        return nvfp4_weights_scaling_factor_2_from_quantizer(wq)
    if not isinstance(wq, SequentialQuantizer) or not wq[-1].is_enabled:
        return None
    assert len(wq) == 2, "modelopt only supports 2 sequential quantization layers for now"
    return get_scaling_factor(wq[-1])


def get_prequant_scaling_factor(module):
    iq = getattr(module, "input_quantizer", None)
    pqs = iq._pre_quant_scale.squeeze() if iq is not None and hasattr(iq, "_pre_quant_scale") else None
    if pqs is not None:
        assert torch.all(pqs > 0), f"prequant scaling factor {pqs} not positive."
    return pqs


# ---- packing (HIP export kernels) --------------------------------------------------------------
def mxfp4_quantize(weight: torch.Tensor, block_size: int | None):
    """MXFP4QTensor.quantize: (packed codes [..., K/2] uint8, E8M0 bytes [n/block, 1] uint8)."""
    return _ops().export_mxfp4(weight, block_size or 32)


def pack_int4_in_uint8(weight, weights_scaling_factor):
    out_dim = weight.shape[-2]
    assert out_dim % 2 == 0, f"Cannot pack weight. Out dimension {out_dim} is not an even number."
    if weight.dim() == 3:
        return torch.stack([_ops().export_int4(w, s) for w, s in zip(weight, weights_scaling_factor)])
    return _ops().export_int4(weight, weights_scaling_factor)


def to_quantized_weight(weight, weights_scaling_factor, quantization, weights_scaling_factor2=None, block_size=None):
    """reference :836-938."""
    if weights_scaling_factor is not None:
        weights_scaling_factor = weights_scaling_factor.to(weight.device)
    if weights_scaling_factor2 is not None:
        weights_scaling_factor2 = weights_scaling_factor2.to(weight.device)
    ops = _ops()
    if quantization == QUANTIZATION_FP8:
        if weight.dtype == torch.float8_e4m3fn:
            warnings.warn("Skipping quantization: weight already in fp8 format")
            return weight
        if weight.dim() == 3:
            return torch.stack([ops.export_fp8(w, s, False, True) for w, s in zip(weight, weights_scaling_factor.reshape(-1))])
        # bf16 / 0-dim fp32 stays in the weight dtype in torch, then casts to e4m3
        return ops.export_fp8(weight, weights_scaling_factor, False, weights_scaling_factor.dim() == 0)
    if quantization in (QUANTIZATION_INT8_SQ, QUANTIZATION_INT8_WO):
        return (weight / weights_scaling_factor[:, None]).round().clamp(-128, 127).to(torch.int8)
    if quantization == QUANTIZATION_FP8_PB_WO:
        # FP8QTensor.quantize with {-1: bs, -2: bs} blocks (reference :874-877): the 2D-block
        # packer divides by the scale of the weight's (row block, column block)
        from ..quantization.qtensor import FP8QTensor

        return FP8QTensor.quantize(
            weight, weights_scaling_factor.squeeze(), block_sizes={-1: block_size, -2: block_size}
        )[0]._quantized_data
    if quantization == QUANTIZATION_FP8_PC_PT:
        if weight.dim() == 3:
            # per-expert scales (reference :880-906): [E] -> [E, 1, 1]; [E, C] matched against the
            # input (BMM-style, [E, 1, K]) or the output dimension ([E, N, 1])
            if weights_scaling_factor.dim() == 1:
                return (weight / weights_scaling_factor[:, None, None]).to(torch.float8_e4m3fn)
            if weights_scaling_factor.dim() == 2:
                if weights_scaling_factor.shape[0] != weight.shape[0]:
                    raise ValueError(
                        "First dimension (num_experts) mismatch for FP8_PC_PT quantization. "
                        f"weight shape: {weight.shape}, scale shape: {weights_scaling_factor.shape}")
                if weight.shape[-1] == weight.shape[-2]:
                    raise ValueError(
                        "Ambiguous scaling dimension for FP8_PC_PT quantization with square weight matrix. "
                        f"weight shape: {weight.shape}, scale shape: {weights_scaling_factor.shape}. "
                        "Cannot determine if scaling should be applied to input_dim or output_dim.")
                if weights_scaling_factor.shape[-1] == weight.shape[-1]:
                    return (weight / weights_scaling_factor.unsqueeze(-2)).to(torch.float8_e4m3fn)
                if weights_scaling_factor.shape[-1] == weight.shape[-2]:
                    return (weight / weights_scaling_factor.unsqueeze(-1)).to(torch.float8_e4m3fn)
                raise ValueError(
                    "Cannot determine correct unsqueeze dimension for FP8_PC_PT quantization. "
                    f"weight shape: {weight.shape}, scale shape: {weights_scaling_factor.shape}")
            return (weight / weights_scaling_factor[:, None]).to(torch.float8_e4m3fn)  # reference :907
        return ops.export_fp8(weight, weights_scaling_factor, True, False)
    if quantization in (QUANTIZATION_INT4_AWQ, QUANTIZATION_W4A8_AWQ):
        return pack_int4_in_uint8(weight, weights_scaling_factor)
    if quantization in NVFP4_FAMILY:
        assert block_size is not None, "Block size not passed. Unable to quantize to NVFP4 format."
        assert weights_scaling_factor2 is not None, "Weights scaling factor 2 not passed."
        s2 = weights_scaling_factor2
        if s2.dim() != 0 and weight.dim() == 3:
            return torch.stack([
                ops.export_nvfp4(w, bs.to(torch.float32), g) for w, bs, g in zip(weight, weights_scaling_factor, s2.reshape(-1))
            ])
        return ops.export_nvfp4(weight, weights_scaling_factor.to(torch.float32), s2)
    if quantization in (QUANTIZATION_W4A8_MXFP4_FP8, QUANTIZATION_MXFP4):
        return mxfp4_quantize(weight, block_size)[0]
    if quantization == QUANTIZATION_MXFP8:
        # MXFP8QTensor.quantize_with_scale (reference :871-872): the HIP packer recomputes the
        # same E8M0 scale from the weight; a scale from elsewhere takes the tensor expression
        from ..quantization.qtensor import MXFP8QTensor

        if weight.dtype not in (torch.bfloat16, torch.float16):  # the packer takes 16-bit weights
            return MXFP8QTensor.quantize_with_scale(weight, weights_scaling_factor)
        q, s = ops.export_mxfp8(weight)
        if weights_scaling_factor is not None and not torch.equal(s, weights_scaling_factor.reshape(s.shape)):
            q = MXFP8QTensor.quantize_with_scale(weight, weights_scaling_factor)
        return q
    raise NotImplementedError(f"quantization format {quantization} not supported")


# ---- fusion preprocessing -------------------------------------------------------------------------
def _recollect_weight_amax(module):
    module.weight_quantizer.reset_amax()
    enable_stats_collection(module.weight_quantizer)
    module.weight_quantizer(module.weight)
    finish_stats_collection(module.weight_quantizer)


def _update_pre_quant_scale(module, new_pqs):
    """W <- W * old / new in fp32, then re-collect the weight amax (reference :1285-1302)."""
    old = module.input_quantizer._pre_quant_scale
    dtype = module.weight.dtype
    module.weight = nn.Parameter(
        (module.weight.to(torch.float32) * old.to(dtype=torch.float32, device=module.weight.device)
         / new_pqs.to(dtype=torch.float32, device=module.weight.device)).to(dtype)
    )
    module.input_quantizer.pre_quant_scale = new_pqs
    _recollect_weight_amax(module)


def preprocess_linear_fusion(modules: list[nn.Module], resmooth_only=False):
    """Average pre_quant_scales, unify input / weight amax of linears fed by one tensor
    (reference :1475-1547)."""
    fmts = [get_quantization_format(m) for m in modules]
    assert all(f == fmts[0] for f in fmts), "Modules have different quantization formats"
    if hasattr(modules[0], "input_quantizer"):
        if modules[0].input_quantizer.pre_quant_scale is not None:
            avg = _mean0([m.input_quantizer.pre_quant_scale for m in modules])
            for m in modules:
                if not torch.equal(m.input_quantizer.pre_quant_scale, avg):
                    _update_pre_quant_scale(m, avg)
        if resmooth_only:
            return
        iq = modules[0].input_quantizer
        if iq.is_enabled and iq.amax is not None:
            assert iq.amax.numel() == 1, "Only support scalar input quant amax"
            input_amax = torch.max(torch.stack([m.input_quantizer.amax for m in modules]))
            for m in modules:
                m.input_quantizer.amax = input_amax
    if hasattr(modules[0], "weight_quantizer"):
        wq = modules[0].weight_quantizer
        if isinstance(wq, SequentialQuantizer):
            if wq[-1].is_enabled:
                assert len(wq) == 2
                amax = torch.max(torch.stack([m.weight_quantizer[-1].amax for m in modules]))
                for m in modules:
                    m.weight_quantizer[-1].amax = amax
        elif isinstance(wq, StaticBlockScaleQuantizer) and wq.is_nvfp4_static:
            gl = [m.weight_quantizer.global_amax for m in modules if m.weight_quantizer.global_amax is not None]
            if gl:
                g = torch.max(torch.stack(gl))
                for m in modules:
                    m.weight_quantizer.global_amax = g
        elif wq.is_enabled and wq.amax is not None and wq.amax.numel() == 1:
            amax = torch.max(torch.stack([m.weight_quantizer.amax for m in modules]))
            for m in modules:
                m.weight_quantizer.amax = amax


def _layernorm_uses_weight_plus_one(module) -> bool:
    if any(n in type(module).__name__ for n in ["LayerNorm1P", "GemmaRMSNorm", "Gemma2RMSNorm", "Gemma3RMSNorm"]):
        return True
    return bool(getattr(module, "zero_centered_gamma", False))


def fuse_prequant_layernorm(layernorm, modules):
    """Fold the (shared) pre_quant_scale into the preceding norm's weight (reference :1442-1472)."""
    if not hasattr(modules[0].input_quantizer, "_pre_quant_scale"):
        return
    pqs = modules[0].input_quantizer._pre_quant_scale.to(layernorm.weight.device)
    if _layernorm_uses_weight_plus_one(layernorm):
        fused = (layernorm.weight + 1.0) * pqs - 1.0
    else:
        fused = layernorm.weight * pqs
    layernorm.weight = nn.Parameter(fused.to(layernorm.weight.dtype))
    if getattr(layernorm, "bias", None) is not None:
        layernorm.bias = nn.Parameter(layernorm.bias * pqs)
    for m in modules:
        delattr(m.input_quantizer, "_pre_quant_scale")
        m.fused_with_prequant = True


# o_proj's / down_proj's pre_quant_scale folds into v_proj's / up_proj's output rows (:1340-1351)
PQS_FUSE_MODULE_MAPPING = [
    (["LlamaAttention", "Qwen3Attention", "Qwen3MoeAttention"], ("v_proj", "o_proj")),
    (["LlamaMLP", "Qwen3MLP", "Qwen3MoeMLP"], ("up_proj", "down_proj")),
]


def fuse_prequant_to_linear(model: nn.Module, fuse_grouped_heads=False):
    """reference :1354-1429 (NVFP4-AWQ)."""
    for _, module in model.named_modules():
        for targets, (into_name, from_name) in PQS_FUSE_MODULE_MAPPING:
            if not any(t in type(module).__name__ for t in targets):
                continue
            into, frm = module.get_submodule(into_name), module.get_submodule(from_name)
            if not (hasattr(frm, "input_quantizer") and hasattr(frm.input_quantizer, "_pre_quant_scale")):
                continue
            pqs = frm.input_quantizer._pre_quant_scale
            if pqs.numel() != into.weight.shape[-2]:
                if not fuse_grouped_heads or "attention" not in type(module).__name__.lower():
                    warnings.warn(f"Skipping pattern fuse prequant for {type(module).__name__}")
                    continue
                nkv = module.config.num_key_value_heads
                hd = into.weight.shape[0] // nkv
                n_rep = pqs.numel() // nkv // hd
                v = pqs.view(nkv, n_rep, hd)
                avg = _mean0([v[:, j] for j in range(n_rep)])
                _update_pre_quant_scale(frm, avg.unsqueeze(1).expand(nkv, n_rep, hd).reshape(-1))
                pqs = avg.reshape(-1)
            into.weight = nn.Parameter(into.weight * pqs.view(-1, 1))
            if getattr(into, "bias", None) is not None:
                into.bias = nn.Parameter(into.bias * pqs)
            _recollect_weight_amax(into)
            delattr(frm.input_quantizer, "_pre_quant_scale")
            frm.fused_with_prequant = True


# ---- config --------------------------------------------------------------------------------------
def _prefix_wildcard_summarize_exclude_modules(unquantized_layers, quantized_layers):
    """Shortest prefix wildcards covering the unquantized layers and no quantized one (:606-677)."""

    def all_prefix_wildcards(name):
        return {name} | {name[:i] + "*" for i in range(len(name) + 1)}

    def formatted_candidates(name):
        for i, ch in enumerate(name):
            if ch == ".":
                yield [name[:i] + "*"]
                yield [name[:i], name[:i] + ".*"]
        yield [name]

    negative = set()
    for layer in quantized_layers:
        negative |= all_prefix_wildcards(layer)
    res = set()
    for layer in unquantized_layers:
        cand = []
        for wildcards in formatted_candidates(layer):
            if any(w in negative for w in wildcards):
                continue
            if all(w in res for w in wildcards):
                cand = []
                break
            cand = wildcards
            break
        if len(cand) == 2:
            a, b = sorted(cand, key=len)
            if b == a + ".*":
                res.add(b)
            else:
                res.update(cand)
        else:
            res.update(cand)
    return res


_ALGO_OF_FORMAT = {
    "fp8": {"quant_algo": "FP8"},
    "fp8_pc_pt": {"quant_algo": "FP8_PER_CHANNEL_PER_TOKEN"},
    "int8_wo": {"quant_algo": "W8A16"},
    "int8_sq": {"quant_algo": "W8A8_SQ_PER_CHANNEL"},
}


def _layer_config(fmt, block_size):
    if fmt in _ALGO_OF_FORMAT:
        return dict(_ALGO_OF_FORMAT[fmt])
    awq = {"has_zero_point": False, "pre_quant_scale": True}
    table = {
        "int4_awq": {"quant_algo": "W4A16_AWQ", "group_size": block_size, **awq},
        "w4a8_awq": {"quant_algo": "W4A8_AWQ", "group_size": block_size, **awq},
        "nvfp4": {"quant_algo": "NVFP4", "group_size": block_size},
        "nvfp4_static": {"quant_algo": "NVFP4", "group_size": block_size},
        "w4a16_nvfp4": {"quant_algo": "W4A16_NVFP4", "group_size": block_size},
        "nvfp4_awq": {"quant_algo": "NVFP4_AWQ", "group_size": block_size, **awq},
        "w4a8_nvfp4_fp8": {"quant_algo": "W4A8_NVFP4_FP8", "group_size": block_size},
        "w4a8_mxfp4_fp8": {"quant_algo": "W4A8_MXFP4_FP8", "group_size": block_size},
        "nvfp4_svdquant": {"quant_algo": "NVFP4_SVD", "group_size": block_size, **awq},
        "mxfp8": {"quant_algo": "MXFP8", "group_size": block_size},
    }
    return table.get(fmt, {"quant_algo": fmt})


def process_layer_quant_config(layer_config_dict: dict) -> dict:
    """Per-layer formats -> the checkpoint's quantization section (reference :680-789)."""
    out: dict[str, Any] = {"quant_algo": None, "kv_cache_quant_algo": None, "quantized_layers": {}}
    formats, cfg, exclude = set(), None, []
    for k, v in layer_config_dict.items():
        if "awq_block_size" in k:
            continue
        prefix = ".".join(k.rsplit(".", 1)[:-1])
        lc = _layer_config(v, layer_config_dict.get(prefix + ".awq_block_size", 0))
        if lc["quant_algo"] != QUANTIZATION_NONE:
            formats.add(str(lc))
            cfg = lc
            out["quantized_layers"][prefix] = lc
        else:
            exclude.append(prefix)
    if len(formats) > 1:
        out["quant_algo"] = "MIXED_PRECISION"
    elif len(formats) == 1 and cfg is not None:
        out.update(cfg)
        out["exclude_modules"] = sorted(
            _prefix_wildcard_summarize_exclude_modules(exclude, out["quantized_layers"].keys())
        )
        out.pop("quantized_layers")
    return out


def _kv_cache_dtype(module) -> str | None:
    """reference :408-462 (FP8 / NVFP4 KV cache from the k/v bmm or output quantizers)."""
    qs = [getattr(module, n) for n in ("k_bmm_quantizer", "v_bmm_quantizer", "output_quantizer")
          if getattr(module, n, None) is not None and getattr(module, n).is_enabled]
    for q in qs:
        if q.num_bits == (4, 3):
            return KV_CACHE_FP8
        if q.num_bits == (2, 1):
            bias = getattr(q, "bias", None)
            return KV_CACHE_NVFP4_AFFINE if bias else KV_CACHE_NVFP4
        if q.num_bits == 8:
            return "INT8"
    return None


def _unquantized_moe_router_names(model) -> list[str]:
    """transformers-5 routers (not nn.Linear, no quantizer) are excluded explicitly (:1550-1580)."""
    names = []
    for name, m in model.named_modules():
        if type(m).__name__.endswith("TopKRouter") or (
            name.endswith(".gate") and hasattr(m, "weight") and not isinstance(m, QuantModule)
            and hasattr(m, "top_k")
        ):
            names.append(name)
    return names


def get_quant_config(model: nn.Module) -> dict[str, Any]:
    """hf_quant_config.json content (reference :1583-1705)."""
    from modelopt_amd import __version__

    cfg: dict[str, Any] = {
        "producer": {"name": "modelopt", "version": __version__},
        "quantization": {"quant_algo": None, "kv_cache_quant_algo": None},
    }
    layer_cfg: dict[str, Any] = {}
    kv_fmt = QUANTIZATION_NONE
    for name, module in dict(model.named_modules()).items():
        wnames = list(weight_attr_names(module))
        has_q = any(
            hasattr(module, quantizer_attr_names(w).weight_quantizer)
            or hasattr(module, quantizer_attr_names(w).input_quantizer)
            or hasattr(module, quantizer_attr_names(w).weight_quantizer + "s")
            for w in wnames
        )
        if has_q:
            fmt = get_quantization_format(module)
            block = 0
            for w in wnames:
                b = get_weight_block_size(module, w)
                if b > 0:
                    block = b
                    break
            if fmt == QUANTIZATION_NVFP4:
                wq = None
                for w in wnames:
                    wq = representative_weight_quantizer(module, w)
                    if wq is not None:
                        break
                if isinstance(wq, StaticBlockScaleQuantizer) and wq.is_nvfp4_static:
                    fmt = "nvfp4_static"
            layer_cfg[name + ".quantization"] = fmt
            layer_cfg[name + ".awq_block_size"] = block
        kv = _kv_cache_dtype(module) if not isinstance(module, QuantModule) or hasattr(module, "k_bmm_quantizer") else None
        if kv is not None:
            if kv_fmt == QUANTIZATION_NONE:
                kv_fmt = kv
            else:
                assert kv_fmt == kv, "Do not support mixed precision kv cache quantization"
    for r in _unquantized_moe_router_names(model):
        layer_cfg.setdefault(r + ".quantization", QUANTIZATION_NONE)
    cfg["quantization"].update(process_layer_quant_config(layer_cfg))
    if kv_fmt is not None:
        cfg["quantization"]["kv_cache_quant_algo"] = kv_fmt
    return cfg


# ---- state dict ------------------------------------------------------------------------------------
_KV_CACHE_REPLACEMENTS = {
    "k_bmm_quantizer._amax": "k_proj.k_scale",
    "v_bmm_quantizer._amax": "v_proj.v_scale",
    "k_bmm_quantizer._bias_value": "k_proj.k_bias",
    "v_bmm_quantizer._bias_value": "v_proj.v_bias",
    "input_quantizer._pre_quant_scale": "pre_quant_scale",
}
_BASE_SKIP_KEYS = ("output_quantizer", "_amax", "_bias_value", "input_quantizer._pre_quant_scale", "weight_shape")


def postprocess_state_dict(state_dict: dict, maxbound: float, kv_cache_format: str | None) -> dict:
    """Drop quantizer state, rename pre-quant / KV scales (reference :1054-1275)."""
    out = {}
    for key, value in state_dict.items():
        if all(sk not in key for sk in _BASE_SKIP_KEYS):
            out[key] = value
            continue
        for old, new in _KV_CACHE_REPLACEMENTS.items():
            if key.endswith(old):
                prefix = key[: -len(old)]
                if "_amax" in key:
                    assert kv_cache_format in (KV_CACHE_FP8, KV_CACHE_NVFP4, KV_CACHE_NVFP4_AFFINE), (
                        "Invalid KV cache quantization format."
                    )
                    value = _div(value.float(), maxbound)  # true division (CPU reference rounding)
                out[prefix + new] = value
                break
    # squeeze (1, n, m) scales
    for k, v in list(out.items()):
        if "scale" in k and isinstance(v, torch.Tensor) and v.dim() == 3 and v.shape[0] == 1:
            out[k] = v.squeeze(0)
    # drop parameters tied to another (same storage) key, keep the first
    seen = {}
    for k in list(out):
        v = out[k]
        if isinstance(v, torch.Tensor) and v.numel() > 0:
            key = (v.untyped_storage().data_ptr(), v.storage_offset(), tuple(v.shape), v.dtype)
            if key in seen and "weight" in k:
                del out[k]
                continue
            seen[key] = k
    return out


__all__ = [
    "get_activation_scaling_factor",
    "get_prequant_scaling_factor",
    "get_quant_config",
    "get_quantization_format",
    "get_scaling_factor",
    "get_weight_block_size",
    "get_weight_scaling_factor",
    "get_weight_scaling_factor_2",
    "postprocess_state_dict",
    "preprocess_linear_fusion",
    "process_layer_quant_config",
    "to_quantized_weight",
]
