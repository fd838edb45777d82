"""``config.json`` ``quantization_config`` in the compressed-tensors layout (reference:
export/convert_hf_config.py:22-276)."""

from __future__ import annotations

import warnings
from collections import defaultdict
from typing import Any

__all__ = ["convert_hf_quant_config_format"]

_F8 = {"dynamic": False, "num_bits": 8, "type": "float"}


def _group_config(quant_algo: str, group_size: int | None = None) -> dict[str, Any]:
    """Per-algorithm ``config_groups`` entry (reference :22-128)."""

    def fp4(gs):
        return {"dynamic": False, "num_bits": 4, "type": "float", "group_size": gs}

    if quant_algo == "FP8":
        return {"input_activations": dict(_F8), "weights": dict(_F8)}
    if quant_algo == "FP8_PER_CHANNEL_PER_TOKEN":
        return {"input_activations": dict(_F8), "weights": {**_F8, "strategy": "channel"}}
    if quant_algo == "NVFP4":
        return {"input_activations": fp4(group_size or 16), "weights": fp4(group_size or 16)}
    if quant_algo == "W4A16_AWQ":
        return {"weights": {"dynamic": False, "num_bits": 4, "type": "int", "group_size": group_size or 128}}
    if quant_algo == "W4A16_NVFP4":
        return {"weights": fp4(group_size or 16)}
    if quant_algo == "NVFP4_SVD":
        gs = group_size or 16
        return {"input_activations": fp4(gs), "weights": fp4(gs), "has_zero_point": False, "pre_quant_scale": True}
    if quant_algo in ("NVFP4_AWQ", "W4A8_AWQ"):
        gs = group_size or 128
        return {"input_activations": {**_F8, "group_size": gs}, "weights": fp4(gs)}
    if quant_algo == "W8A16":
        return {"weights": {"dynamic": False, "num_bits": 8, "type": "int"}}
    if quant_algo == "W8A8_SQ_PER_CHANNEL":
        return {
            "input_activations": {"dynamic": False, "num_bits": 8, "type": "int"},
            "weights": {"dynamic": False, "num_bits": 8, "type": "int", "strategy": "channel"},
        }
    if quant_algo in ("W4A8_NVFP4_FP8", "W4A8_MXFP4_FP8"):
        return {"input_activations": dict(_F8), "weights": fp4(group_size or 16)}
    if quant_algo == "MXFP8":
        gs = group_size or 32
        return {"input_activations": {**_F8, "group_size": gs}, "weights": {**_F8, "group_size": gs}}
    warnings.warn(f"Unsupported quantization algorithm '{quant_algo}' in the config-group mapping.")
    return {"quant_algo": quant_algo}


def convert_hf_quant_config_format(input_config: dict[str, Any]) -> dict[str, Any]:
    """hf_quant_config -> llm-compressor style ``quantization_config`` (reference :130-276)."""
    new: dict[str, Any] = {}
    q = input_config.get("quantization", {})
    algo = q.get("quant_algo")
    single = {"FP8", "NVFP4", "W4A16_NVFP4", "NVFP4_SVD"}
    if algo in single:
        grp = _group_config(algo, q.get("group_size"))
        if algo == "NVFP4_SVD" and q.get("lora_rank") is not None:
            grp["lora_rank"] = q["lora_rank"]
        grp["targets"] = ["Linear"]
        new["config_groups"] = {"group_0": grp}
    elif algo == "MIXED_PRECISION":
        layers = q.get("quantized_layers", {})
        by_cfg: dict[tuple, list[str]] = defaultdict(list)
        for name, lc in layers.items():
            by_cfg[tuple(sorted(lc.items()))].append(name)
        groups = {}
        for i, (key, names) in enumerate(by_cfg.items()):
            lc = dict(key)
            g = _group_config(lc.get("quant_algo", ""), lc.get("group_size"))
            g["targets"] = sorted(names)
            groups[f"group_{i}"] = g
        new["config_groups"] = groups
        new["quantized_layers"] = layers
    excl = q.get("exclude_modules")
    new["ignore"] = excl if excl is not None else []
    if algo:
        new["quant_algo"] = algo
    kv = q.get("kv_cache_quant_algo")
    if kv:
        new["kv_cache_scheme"] = dict(_F8) if kv == "FP8" else kv
    if input_config.get("producer"):
        new["producer"] = input_config["producer"]
    new["quant_method"] = "modelopt"
    return new
