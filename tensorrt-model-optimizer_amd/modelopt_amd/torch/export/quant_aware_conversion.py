"""Map exported tensor names back to the hub checkpoint's (reference: export/quant_aware_conversion.py).

transformers >= 5 may rename / fuse weights at load time (``conversion_mapping``: Mixtral's
``block_sparse_moe`` -> ``mlp``, per-expert ``w1``/``w3`` -> stacked ``gate_up_proj``, ...).
Its own ``revert_weight_conversion`` cannot handle quantized state dicts (0-d scale tensors), so
export reverses the mapping here while carrying every weight's scale siblings along:

* ``WeightRenaming``                  -> regex key renames (scales share the module prefix);
* expert ``WeightConverter`` (reverse has ``SplitModulelist``) -> per-expert leaf renames, since
  export already expanded the experts into ``experts.<i>.{gate,up,down}_proj``;
* dense fusing converter (reverse is ``Chunk`` only) -> split of the fused tensors along dim 0,
  per-tensor scalar scales duplicated.

Anything else raises :class:`QuantConversionUnsupportedError` and the caller keeps the in-memory
names for both weights and config.
"""

from __future__ import annotations

import re
from dataclasses import dataclass

import torch

__all__ = [
    "QuantConversionUnsupportedError",
    "build_reverse_name_mapper",
    "revert_quant_config_names",
    "revert_weight_conversion_quant_aware",
]

_LEAVES = (".weight", ".weight_scale", ".weight_scale_2", ".weight_scale_inv", ".input_scale", ".bias")
_SCALAR_LEAVES = (".weight_scale_2", ".input_scale")
_EXPERT_PARTS = {"gate_up_proj": ["gate_proj", "up_proj"]}


class QuantConversionUnsupportedError(Exception):
    """The conversion mapping uses an op that cannot be reversed with the scales attached."""


@dataclass(frozen=True)
class _Rename:
    pattern: str
    repl: str
    scopes: tuple = ()


@dataclass(frozen=True)
class _Split:
    fused: str
    parts: tuple
    dim: int = 0


def _as_list(x):
    return list(x) if isinstance(x, (list, tuple)) else [x]


def _leaf(pattern: str) -> str:
    p = pattern.removesuffix(".weight")
    return p.rsplit(".", 1)[-1]


def _scopes(rev) -> tuple:
    scope = getattr(rev, "scope_prefix", None)
    if scope is None:
        return ()
    s = f"{scope}." if scope else ""
    base = getattr(rev, "base_model_prefix", None) or ""
    b = f"{base}." if base else ""
    out = []
    for c in (b + s, s):
        if c not in out:
            out.append(c)
    return tuple(out)


def _build_rules(model):
    try:
        conversions = getattr(model, "_weight_conversions", None)
        if conversions is None:
            from transformers.conversion_mapping import get_model_conversion_mapping

            conversions = get_model_conversion_mapping(model, add_legacy=False)
        from transformers.core_model_loading import Chunk, SplitModulelist, WeightConverter, WeightRenaming
    except Exception as exc:  # noqa: BLE001 -- transformers without the API
        raise QuantConversionUnsupportedError(f"could not read conversion mapping: {exc}") from exc
    if not conversions:
        return [], [], []
    splits, renames, leaf_renames, fused_leaves = [], [], [], []
    for conv in conversions:
        rev = conv.reverse_transform()
        if isinstance(rev, WeightRenaming):
            for p, r in zip(_as_list(rev.source_patterns), _as_list(rev.target_patterns)):
                renames.append(_Rename(p, r, _scopes(rev)))
        elif isinstance(rev, WeightConverter):
            if _scopes(rev):
                raise QuantConversionUnsupportedError("scoped WeightConverter")
            ops = list(rev.operations)
            if any(isinstance(o, SplitModulelist) for o in ops):
                src = _leaf(_as_list(rev.source_patterns)[0])
                hubs = [_leaf(t) for t in _as_list(rev.target_patterns)]
                parts = _EXPERT_PARTS.get(src, [src])
                if len(parts) != len(hubs):
                    raise QuantConversionUnsupportedError(f"expert arity {parts} vs {hubs}")
                for part, hub in zip(parts, hubs):
                    leaf_renames.append(_Rename(rf"(\.experts\.\d+\.){re.escape(part)}\b", rf"\g<1>{hub}"))
                fused_leaves.append(src)
            elif ops and all(isinstance(o, Chunk) for o in ops):
                src = _as_list(rev.source_patterns)[0].removesuffix(".weight")
                parts = tuple("." + _leaf(t) for t in _as_list(rev.target_patterns))
                splits.append(_Split("." + _leaf(src), parts, 0))
            else:
                raise QuantConversionUnsupportedError(f"unsupported reverse ops {[type(o).__name__ for o in ops]}")
        else:
            raise QuantConversionUnsupportedError(f"unsupported conversion {type(rev).__name__}")
    # converters first, then renamings in reverse list order (transformers' save path)
    return splits, leaf_renames + list(reversed(renames)), fused_leaves


def _sub(rule, compiled, key):
    if not rule.scopes:
        return compiled.sub(rule.repl, key)
    for prefix in rule.scopes:
        if key.startswith(prefix):
            return prefix + compiled.sub(rule.repl, key[len(prefix):])
    return key


def _rename_fn(renames):
    compiled = [(r, re.compile(r.pattern)) for r in renames]

    def apply(key):
        for r, c in compiled:
            key = _sub(r, c, key)
        return key

    return apply


def revert_weight_conversion_quant_aware(model, state_dict: dict) -> dict:
    splits, renames, fused_leaves = _build_rules(model)
    if not splits and not renames:
        return state_dict
    if fused_leaves:
        pat = re.compile(r"\.experts\.(?:" + "|".join(map(re.escape, fused_leaves)) + r")(?:\.|$)")
        for k, v in state_dict.items():
            if pat.search(k) or (".experts." in k and getattr(v, "ndim", 0) >= 3):
                raise QuantConversionUnsupportedError(f"experts not pre-expanded ({k})")
    out = dict(state_dict)
    for rule in splits:
        hits = [(k[: -len(leaf)][: -len(rule.fused)], leaf, k) for k in list(out) for leaf in _LEAVES
                if k.endswith(rule.fused + leaf)]
        for module, leaf, key in hits:
            t = out.pop(key)
            n = len(rule.parts)
            for i, part in enumerate(rule.parts):
                tgt = module + part + leaf
                if tgt in out:
                    raise QuantConversionUnsupportedError(f"split collision on {tgt}")
                if leaf in _SCALAR_LEAVES or t.dim() == 0:
                    out[tgt] = t.clone()
                else:
                    if t.size(rule.dim) % n:
                        raise QuantConversionUnsupportedError(f"cannot split {key}")
                    out[tgt] = t.chunk(n, dim=rule.dim)[i].clone()
    apply = _rename_fn(renames)
    renamed = {}
    for k, v in out.items():
        nk = apply(k)
        if nk in renamed:
            raise QuantConversionUnsupportedError(f"rename collision on {nk}")
        renamed[nk] = v
    return renamed


def build_reverse_name_mapper(model):
    """Module-name mapper for the config's exclude / quantized-layer names (reference :236-276)."""
    _, renames, _ = _build_rules(model)
    if not renames:
        return None
    apply = _rename_fn(renames)
    sentinel = ".\x00modelopt_name_sentinel"

    def mapper(name: str) -> str:
        base, suffix = name, ""
        if name.endswith(".*"):
            base, suffix = name[:-2], ".*"
        elif name.endswith("*"):
            base, suffix = name[:-1], "*"
        return apply(base + sentinel).removesuffix(sentinel) + suffix

    return mapper


def revert_quant_config_names(quantization: dict, mapper) -> None:
    if mapper is None or not isinstance(quantization, dict):
        return
    if quantization.get("exclude_modules"):
        quantization["exclude_modules"] = [mapper(e) for e in quantization["exclude_modules"]]
    ql = quantization.get("quantized_layers")
    if isinstance(ql, dict) and ql:
        quantization["quantized_layers"] = {mapper(k): v for k, v in ql.items()}


_ = torch
