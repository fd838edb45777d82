"""Quantizer attribute / quantize configs and the preset configs of the hot path.

Mirrors the schema of modelopt/torch/quantization/config.py: ``QuantizerAttributeConfig``
(:322-709), ``QuantizerCfgEntry`` (:165-243) with its normalisation rules, ``QuantizeConfig``
(:1573), the calibration-algorithm configs used on the PTQ path (``MaxCalibConfig`` :894,
``AWQLiteCalibConfig`` :1084), and the preset dicts (``INT8_DEFAULT_CFG`` ... :1681-1778) that the
reference composes from ``modelopt_recipes/configs/ptq/...`` YAML units.  The presets here are
written out as plain dicts with the same entries (no YAML loader on the hot path).
"""

from __future__ import annotations

import copy
import re
from collections.abc import Callable, Mapping
from typing import Any

from pydantic import BaseModel, ConfigDict, Field, ValidationInfo, field_validator, model_validator

__all__ = [
    "AWQClipCalibConfig",
    "AWQFullCalibConfig",
    "AWQLiteCalibConfig",
    "LayerwiseConfig",
    "MaxCalibConfig",
    "MseCalibConfig",
    "find_quant_cfg_entry_by_path",
    "QuantizeAlgorithmConfig",
    "QuantizeConfig",
    "QuantizerAttributeConfig",
    "QuantizerCfgEntry",
    "choices",
    "need_calibration",
    "normalize_quant_cfg_list",
]


class _Config(BaseModel):
    """Pydantic base with the dict-like accessors the reference's ModeloptBaseConfig offers."""

    model_config = ConfigDict(extra="forbid", validate_assignment=True, arbitrary_types_allowed=True)

    def items(self):
        return self.model_dump().items()

    def keys(self):
        return self.model_dump().keys()

    def get(self, key, default=None):
        return getattr(self, key, default)

    def __getitem__(self, key):
        return getattr(self, key)

    def __contains__(self, key):
        return key in type(self).model_fields


_EXMY = re.compile(r"^e(\d+)m(\d+)$", re.IGNORECASE)
_FP_FORMATS = [(4, 3), (5, 2), (2, 1), (1, 2), (0, 3), (3, 0), (3, 2), (2, 3)]


def _parse_num_bits(v):
    if isinstance(v, str):
        m = _EXMY.match(v.strip())
        if m:
            return (int(m.group(1)), int(m.group(2)))
        if v.isdigit():
            return int(v)
        return v
    if isinstance(v, list):
        return tuple(v)
    return v


def _parse_block_sizes(v):
    if v is None:
        return None
    out = {}
    for k, val in dict(v).items():
        if isinstance(k, str) and k.lstrip("-").isdigit():
            k = int(k)
        if k == "scale_bits" and isinstance(val, (list, str)):
            val = _parse_num_bits(val)
        if k == "scale_block_sizes" and isinstance(val, Mapping):
            val = {int(a) if isinstance(a, str) and a.lstrip("-").isdigit() else a: b for a, b in val.items()}
        out[k] = val
    return out


class QuantizerAttributeConfig(_Config):
    """Attributes of one TensorQuantizer (reference config.py:322-709)."""

    enable: bool = True
    num_bits: int | tuple[int, int] | str = 8
    effective_bits: float | None = None
    axis: int | tuple[int, ...] | None = None
    fake_quant: bool = True
    unsigned: bool = False
    narrow_range: bool = False  # reference default False (config.py:459-463)
    learn_amax: bool = False
    type: str = Field(default="static", pattern=r"^static$|^dynamic$")
    block_sizes: dict | None = None
    bias: dict | None = None
    trt_high_precision_dtype: str = Field(default="Float", pattern=r"^Float$|^Half$|^BFloat16$")
    calibrator: Any = "max"
    rotate: Any = False
    pass_through_bwd: bool = True
    backend: str | None = None
    backend_extra_args: dict | None = None
    use_constant_amax: bool = False
    constant_amax: float | None = None

    @model_validator(mode="before")
    @classmethod
    def _validate_config(cls, values):
        if isinstance(values, Mapping):
            values = dict(values)
            if len(values) == 1 and values.get("enable") is True:
                raise ValueError(
                    "Invalid quantizer config: Cannot specify only {'enable': True}. "
                    "Additional parameters are required when enabling quantization."
                )
            if "num_bits" in values:
                values["num_bits"] = _parse_num_bits(values["num_bits"])
            if "block_sizes" in values:
                values["block_sizes"] = _parse_block_sizes(values["block_sizes"])
            if isinstance(values.get("axis"), list):
                values["axis"] = tuple(values["axis"])
        return values

    @field_validator("effective_bits")
    @classmethod
    def _validate_effective_bits(cls, v):
        if v is not None and not (0 < v <= 16):
            raise ValueError(f"effective_bits must be in (0, 16], got {v}")
        return v

    @field_validator("learn_amax")
    @classmethod
    def _validate_learn_amax(cls, v):
        assert v is not True, "learn_amax is deprecated and reserved for backward compatibility."
        return v

    @field_validator("block_sizes")
    @classmethod
    def _validate_block_sizes(cls, v, info: ValidationInfo):
        if v is None:
            return v
        assert info.data.get("axis") is None, "axis must be None when block_sizes is not None."
        if v.get("type", None) == "dynamic":
            assert len(cls._get_block_quant_axes_and_sizes(v)) == 1, (
                "Dynamic block quantization only supports quantization last axis."
            )
        for k, val in v.items():
            if isinstance(k, str):
                assert k in ["type", "scale_bits", "scale_block_sizes", "four_over_six"]
            else:
                assert isinstance(k, int) and (val is None or isinstance(val, int))
        return v

    @field_validator("bias")
    @classmethod
    def _validate_bias(cls, v):
        if v is None:
            return v
        if "type" in v and v["type"] not in ["static", "dynamic"]:
            raise ValueError(f"Invalid bias type: {v['type']}, expected 'static' or 'dynamic'")
        if "method" in v and v["method"] not in ["mean", "max_min"]:
            raise ValueError(f"Invalid bias method: {v['method']}, expected 'mean' or 'max_min'")
        axis = [k for k in v if k not in ["type", "method"]]
        assert len(axis) > 0, "The axis for bias computation is not specified."
        for x in axis:
            if not isinstance(x, int):
                raise ValueError(f"Invalid axis type {type(axis)}, expected int")
        return v

    @field_validator("calibrator")
    @classmethod
    def _validate_calibrator(cls, v):
        if isinstance(v, str):
            assert v in ["max", "histogram"]
        return v

    @field_validator("constant_amax")
    @classmethod
    def _validate_constant_amax(cls, v):
        assert v is None or v > 0, "constant_amax must be a positive value."
        return v

    @model_validator(mode="after")
    def _validate_num_bits(self):
        if self.backend is not None:
            return self
        nb = self.num_bits
        if isinstance(nb, int) and nb < 1:
            raise ValueError(f"num_bits must be a positive integer or a tuple of positive integers. {nb}")
        if isinstance(nb, tuple):
            if not all(x >= 0 for x in nb) or not any(x > 0 for x in nb):
                raise ValueError("num_bits must be a positive integer or a tuple of positive integers.")
            if nb not in _FP_FORMATS:
                raise ValueError(
                    "Supported FPx quantization formats: FP8 (E4M3, E5M2), FP6(E3M2, E2M3), FP4(E2M1)."
                )
            bs = self.block_sizes
            if nb not in [(4, 3), (2, 1)] and (bs is None or bs.get("type", None) != "dynamic"):
                raise ValueError(
                    "Only blockwise dynamic quantization is supported with quantization formats "
                    f"E{nb[0]}M{nb[1]}."
                )
        assert not (self.use_constant_amax and self.constant_amax is not None), (
            "use_constant_amax and constant_amax are mutually exclusive; set only one."
        )
        return self

    @staticmethod
    def _get_block_quant_axes_and_sizes(block_sizes):
        if block_sizes is None:
            return None
        return {
            k: v
            for k, v in block_sizes.items()
            if k not in ["type", "scale_bits", "scale_block_sizes", "four_over_six"]
        }


class QuantizerCfgEntry(_Config):
    """One entry of an ordered ``quant_cfg`` list (reference config.py:165-243)."""

    quantizer_name: str
    parent_class: str | None = None
    cfg: QuantizerAttributeConfig | list[QuantizerAttributeConfig] | None = None
    enable: bool = True

    @model_validator(mode="before")
    @classmethod
    def _normalize_cfg_shape(cls, values):
        if not isinstance(values, dict):
            return values
        cfg = values.get("cfg")
        empty = (isinstance(cfg, dict) and len(cfg) == 0) or (
            isinstance(cfg, list)
            and (len(cfg) == 0 or all(isinstance(i, dict) and len(i) == 0 for i in cfg))
        )
        if empty:
            if values.get("enable") is False:
                values = {**values, "cfg": None}
            else:
                raise ValueError(
                    f"QuantizerCfgEntry 'cfg' must specify at least one quantizer attribute; got an "
                    f"empty mapping/list for quantizer {values.get('quantizer_name')!r}."
                )
        return values

    @model_validator(mode="after")
    def _validate_instruction(self):
        if "cfg" not in self.model_fields_set and "enable" not in self.model_fields_set:
            raise ValueError(
                "QuantizerCfgEntry must specify 'cfg', 'enable', or both "
                f"(quantizer_name={self.quantizer_name!r})."
            )
        return self


def normalize_quant_cfg_list(quant_cfg) -> list[dict[str, Any]]:
    """Normalise a quant_cfg (ordered list of entries, or a legacy {pattern: cfg} dict) to a list of
    ``{"quantizer_name", "parent_class", "cfg", "enable"}`` dicts with explicit ``enable``/``cfg``
    (reference config.py:1447-1571)."""
    if quant_cfg is None:
        return []
    entries: list = []
    if isinstance(quant_cfg, Mapping):
        # legacy dict form: {"*weight_quantizer": {...}, "default": {...}, "nn.Linear": {"*": ...}}
        for k, v in quant_cfg.items():
            if k == "default":
                k = "*"
            if isinstance(v, Mapping) and k.startswith("nn.") and all(isinstance(kk, str) for kk in v):
                for kk, vv in v.items():
                    entries.append(_legacy_entry(kk, vv, parent_class=k))
                continue
            entries.append(_legacy_entry(k, v))
    else:
        entries = list(quant_cfg)
    out = []
    for e in entries:
        if isinstance(e, QuantizerCfgEntry):
            e = {k: getattr(e, k) for k in e.model_fields_set | {"quantizer_name"}}
        e = dict(e)
        QuantizerCfgEntry(**e)  # validate shape
        cfg = e.get("cfg")
        if isinstance(cfg, Mapping) and len(cfg) == 0 and e.get("enable") is False:
            cfg = None
        enable = e.get("enable", True)
        if isinstance(cfg, QuantizerAttributeConfig):
            cfg = {k: getattr(cfg, k) for k in cfg.model_fields_set}
        elif isinstance(cfg, list):
            cfg = [
                {k: getattr(c, k) for k in c.model_fields_set} if isinstance(c, QuantizerAttributeConfig) else dict(c)
                for c in cfg
            ]
        elif isinstance(cfg, Mapping):
            cfg = dict(cfg)
            if "enable" in cfg:  # legacy: enable inside cfg
                enable = cfg.pop("enable") if "enable" not in e else enable
                if not cfg:
                    cfg = None
        out.append(
            {
                "quantizer_name": e["quantizer_name"],
                "parent_class": e.get("parent_class"),
                "cfg": cfg,
                "enable": enable,
            }
        )
    return out


def _legacy_entry(name, v, parent_class=None):
    e: dict[str, Any] = {"quantizer_name": name}
    if parent_class:
        e["parent_class"] = parent_class
    if isinstance(v, Mapping) and set(v.keys()) == {"enable"}:
        e["enable"] = v["enable"]
    else:
        if isinstance(v, Mapping) and "enable" in v:
            v = dict(v)
            e["enable"] = v.pop("enable")
        e["cfg"] = v
    return e


def find_quant_cfg_entry_by_path(quant_cfg_list, quantizer_name: str):
    """The LAST entry of a ``quant_cfg`` list whose ``quantizer_name`` equals ``quantizer_name``
    exactly (no wildcard matching; later entries override earlier ones, so the last one is the
    effective configuration) -- reference config.py:245-276.  KeyError when there is none."""
    found = None
    for entry in quant_cfg_list:
        if entry.get("quantizer_name") == quantizer_name:
            found = entry
    if found is None:
        raise KeyError(f"No quant_cfg entry with quantizer_name={quantizer_name!r}")
    return found


class LayerwiseConfig(_Config):
    """Layer-by-layer calibration options (reference config.py:712-770; ``algorithm["layerwise"]``,
    run by ``layerwise.layerwise_calibrate``)."""

    enable: bool = False
    get_qdq_activations_from_prev_layer: bool = False
    checkpoint_dir: str | None = None
    save_every: int = Field(default=1, ge=1)
    calib_mutates_weights: bool = True


class QuantizeAlgorithmConfig(_Config):
    """Base calibration-algorithm config (reference config.py:780)."""

    model_config = ConfigDict(extra="allow", validate_assignment=True, arbitrary_types_allowed=True)
    method: str | None = None
    # fraction of experts every token is routed to during calibration forwards (reference
    # config.py:793-803; 0 < r <= 1)
    moe_calib_experts_ratio: float | None = Field(default=None, gt=0.0, le=1.0)
    layerwise: Any = None


class MaxCalibConfig(QuantizeAlgorithmConfig):
    method: str | None = "max"
    distributed_sync: bool | None = True
    sync_expert_weight_amax: bool = False
    shared_states: Any = None


class MseCalibConfig(QuantizeAlgorithmConfig):
    """``mse`` weight-amax search (reference config.py:938-998)."""

    method: str | None = "mse"
    step_size: float | None = Field(default=0.1, gt=0.0)
    start_multiplier: float | None = Field(default=0.25, gt=0.0)
    stop_multiplier: float | None = Field(default=4.0, gt=0.0)
    fp8_scale_sweep: bool | None = False
    distributed_sync: bool | None = True
    shared_states: Any = None


class AWQLiteCalibConfig(QuantizeAlgorithmConfig):
    method: str | None = "awq_lite"
    alpha_step: float = Field(default=0.1, gt=0.0, le=1.0)
    debug: bool = False


class AWQClipCalibConfig(QuantizeAlgorithmConfig):
    method: str | None = "awq_clip"
    max_co_batch_size: int = 1024
    max_tokens_per_batch: int = 64
    min_clip_ratio: float = 0.5
    shrink_step: float = 0.05
    debug: bool = False


class AWQFullCalibConfig(AWQLiteCalibConfig, AWQClipCalibConfig):
    method: str | None = "awq_full"


_ALGO_CONFIGS: dict[str, type[QuantizeAlgorithmConfig]] = {
    "max": MaxCalibConfig,
    "mse": MseCalibConfig,
    "awq_lite": AWQLiteCalibConfig,
    "awq_clip": AWQClipCalibConfig,
    "awq_full": AWQFullCalibConfig,
}


def algorithm_config(algorithm) -> QuantizeAlgorithmConfig | None:
    if algorithm is None:
        return None
    if isinstance(algorithm, QuantizeAlgorithmConfig):
        return algorithm
    if isinstance(algorithm, str):
        algorithm = {"method": algorithm}
    algorithm = dict(algorithm)
    method = algorithm.get("method")
    cls = _ALGO_CONFIGS.get(method)
    if cls is None:
        raise NotImplementedError(
            f"modelopt_amd: calibration algorithm {method!r} is outside the MI355X-native hot path "
            "(supported: max, mse, awq_lite, awq_clip, awq_full)"
        )
    return cls(**algorithm)


class QuantizeConfig(_Config):
    """``{"quant_cfg": [...], "algorithm": ...}`` (reference config.py:1573)."""

    quant_cfg: Any = Field(default_factory=list)
    algorithm: Any = "max"

    @field_validator("quant_cfg")
    @classmethod
    def _normalize(cls, v):
        return normalize_quant_cfg_list(v)


def need_calibration(config) -> bool:
    """Whether a config needs a calibration forward (reference config.py:1827)."""
    cfg = config if isinstance(config, Mapping) else config.model_dump()
    algo = cfg.get("algorithm")
    if algo is not None and (algo if isinstance(algo, str) else algo.get("method")) not in (None, "max"):
        return True
    for e in normalize_quant_cfg_list(cfg.get("quant_cfg", [])):
        c = e["cfg"]
        if not e["enable"] or c is None:
            continue
        cs = c if isinstance(c, list) else [c]
        for ci in cs:
            bs = ci.get("block_sizes") or {}
            if ci.get("type", "static") == "static" and bs.get("type", "static") == "static":
                if "input_quantizer" in e["quantizer_name"] or "output_quantizer" in e["quantizer_name"]:
                    return True
    return False


def choices(config: Mapping) -> Mapping:
    return config


# ----------------------------------------------------------------------------------------------
# Presets.  Entry lists equal to the reference's YAML-composed presets
# (modelopt_recipes/configs/ptq/units/{base_disable_all,default_disabled_quantizers}.yaml + the
# per-format numerics units); printed from the reference in SURVEY §8.
# ----------------------------------------------------------------------------------------------

_BASE_DISABLE_ALL = [{"quantizer_name": "*", "enable": False}]

_DEFAULT_DISABLED_QUANTIZERS = [
    {"quantizer_name": n, "enable": False}
    for n in [
        "*block_sparse_moe.gate*",
        "*linear_attn.conv1d*",
        "*linear_attn.in_proj_a*",
        "*linear_attn.in_proj_b*",
        "*lm_head*",
        "*mixer.conv1d*",
        "*mlp.gate.*",
        "*mlp.shared_expert_gate.*",
        "*output_layer*",
        "*proj_out.*",
        "*router*",
        "mtp.*",
        "output.*",
        "*embed_vision*",
        "*vision_tower*",
        "*visual*",
        "*vision_model*",
        "*multi_modal_projector*",
    ]
] + [
    {"quantizer_name": "*", "parent_class": c, "enable": False}
    for c in ["nn.BatchNorm1d", "nn.BatchNorm2d", "nn.BatchNorm3d", "nn.LeakyReLU", "nn.Embedding"]
]


def _preset(weight, inp, algorithm="max") -> dict[str, Any]:
    qc = list(_BASE_DISABLE_ALL)
    if weight is not None:
        qc.append({"quantizer_name": "*weight_quantizer", "cfg": weight})
    if inp is None:
        qc.append({"quantizer_name": "*input_quantizer", "enable": False})
    elif inp != "keep":
        qc.append({"quantizer_name": "*input_quantizer", "cfg": inp})
    qc += _DEFAULT_DISABLED_QUANTIZERS
    return {"quant_cfg": copy.deepcopy(qc), "algorithm": copy.deepcopy(algorithm)}


_MX = lambda nb: {"num_bits": nb, "block_sizes": {-1: 32, "type": "dynamic", "scale_bits": (8, 0)}}  # noqa: E731

INT8_DEFAULT_CFG: dict[str, Any] = _preset({"num_bits": 8, "axis": 0}, {"num_bits": 8, "axis": None})
INT8_WEIGHT_ONLY_CFG: dict[str, Any] = _preset({"num_bits": 8, "axis": 0}, None)
FP8_DEFAULT_CFG: dict[str, Any] = _preset(
    {"num_bits": (4, 3), "axis": None}, {"num_bits": (4, 3), "axis": None}
)
FP8_PER_CHANNEL_PER_TOKEN_CFG: dict[str, Any] = _preset(
    {"num_bits": (4, 3), "axis": 0},
    {"num_bits": (4, 3), "axis": None, "type": "dynamic", "block_sizes": {-1: None}},
)
FP8_2D_BLOCKWISE_WEIGHT_ONLY_CFG: dict[str, Any] = _preset(
    {"num_bits": (4, 3), "axis": None, "block_sizes": {-1: 128, -2: 128}}, None
)
INT4_BLOCKWISE_WEIGHT_ONLY_CFG: dict[str, Any] = _preset(
    {"num_bits": 4, "block_sizes": {-1: 128, "type": "static"}}, None
)
INT4_AWQ_CFG: dict[str, Any] = _preset(
    {"num_bits": 4, "block_sizes": {-1: 128, "type": "static"}},
    None,
    {"method": "awq_lite", "alpha_step": 0.1},
)
MXFP8_DEFAULT_CFG: dict[str, Any] = _preset(_MX((4, 3)), _MX((4, 3)), None)
MXFP6_DEFAULT_CFG: dict[str, Any] = _preset(_MX((3, 2)), _MX((3, 2)), None)
MXFP4_DEFAULT_CFG: dict[str, Any] = _preset(_MX((2, 1)), _MX((2, 1)), None)
MXINT8_DEFAULT_CFG: dict[str, Any] = _preset(_MX(8), _MX(8), None)
W4A8_MXFP4_FP8_CFG: dict[str, Any] = _preset(_MX((2, 1)), {"num_bits": (4, 3), "axis": None}, None)
_NVFP4 = {"num_bits": (2, 1), "effective_bits": 4.5,
          "block_sizes": {-1: 16, "type": "dynamic", "scale_bits": (4, 3)}}
NVFP4_DEFAULT_CFG: dict[str, Any] = _preset(_NVFP4, _NVFP4, "max")
NVFP4_AWQ_LITE_CFG: dict[str, Any] = _preset(_NVFP4, _NVFP4, "awq_lite")
NVFP4_AWQ_CLIP_CFG: dict[str, Any] = _preset(_NVFP4, _NVFP4, {"method": "awq_clip"})
NVFP4_AWQ_FULL_CFG: dict[str, Any] = _preset(_NVFP4, _NVFP4, {"method": "awq_full", "alpha_step": 0.1})
_NVFP4_STATIC = {"num_bits": (2, 1), "block_sizes": {-1: 16, "type": "static", "scale_bits": (4, 3)}}
NVFP4_W4A4_WEIGHT_MSE_FP8_SWEEP_CFG: dict[str, Any] = _preset(
    _NVFP4_STATIC, _NVFP4, {"method": "mse", "fp8_scale_sweep": True}
)
W4A8_AWQ_BETA_CFG: dict[str, Any] = _preset(
    [{"num_bits": 4, "block_sizes": {-1: 128, "type": "static"}}, {"num_bits": (4, 3), "axis": None}],
    {"num_bits": (4, 3), "axis": None},
    "awq_lite",
)
FP8_KV_CFG: dict[str, Any] = {
    "quant_cfg": [{"quantizer_name": "*[kv]_bmm_quantizer", "cfg": {"num_bits": (4, 3), "axis": None}}],
}
NVFP4_KV_CFG: dict[str, Any] = {
    "quant_cfg": [{"quantizer_name": "*[kv]_bmm_quantizer", "cfg": copy.deepcopy(_NVFP4)}],
}
_AFFINE = {"bias": {-2: None, -4: None, "type": "static"}}
FP8_AFFINE_KV_CFG: dict[str, Any] = {
    "quant_cfg": [
        {"quantizer_name": "*[kv]_bmm_quantizer", "cfg": {"num_bits": (4, 3), "axis": None}},
        {"quantizer_name": "*[kv]_bmm_quantizer", "cfg": {"num_bits": (4, 3), "axis": None, **copy.deepcopy(_AFFINE)}},
    ],
}
NVFP4_AFFINE_KV_CFG: dict[str, Any] = {
    "quant_cfg": [
        {"quantizer_name": "*[kv]_bmm_quantizer", "cfg": copy.deepcopy(_NVFP4)},
        {"quantizer_name": "*[kv]_bmm_quantizer", "cfg": {**copy.deepcopy(_NVFP4), **copy.deepcopy(_AFFINE)}},
    ],
}
_FP8_PT = {"num_bits": (4, 3), "axis": None}
NVFP4_FP8_MHA_CONFIG: dict[str, Any] = {
    "quant_cfg": copy.deepcopy(
        _BASE_DISABLE_ALL
        + [
            {"quantizer_name": "*weight_quantizer", "cfg": _NVFP4},
            {"quantizer_name": "*input_quantizer", "cfg": _NVFP4},
            {"quantizer_name": "*output_quantizer", "enable": False},
            {"quantizer_name": "*[qkv]_bmm_quantizer", "cfg": _FP8_PT},
            {"quantizer_name": "*softmax_quantizer", "cfg": _FP8_PT},
            {"quantizer_name": "*p_bmm_quantizer", "cfg": _FP8_PT},
            {"quantizer_name": "transformer_blocks*bmm2_output_quantizer", "cfg": _FP8_PT},
        ]
    ),
    "algorithm": "max",
}
MXFP4_MLP_WEIGHT_ONLY_CFG: dict[str, Any] = {
    "quant_cfg": _BASE_DISABLE_ALL
    + [
        {"quantizer_name": "*mlp*weight_quantizer", "cfg": _MX((2, 1))},
        {"quantizer_name": "*block_sparse_moe*weight_quantizer", "cfg": _MX((2, 1))},
    ]
    + _DEFAULT_DISABLED_QUANTIZERS,
    "algorithm": None,
}

_NVFP4_B32 = {"num_bits": (2, 1), "block_sizes": {-1: 32, "type": "dynamic", "scale_bits": (4, 3)}}
W4A16_NVFP4_CFG: dict[str, Any] = _preset(_NVFP4, "keep")
W4A8_NVFP4_FP8_CFG: dict[str, Any] = _preset(_NVFP4_B32, {"num_bits": (4, 3), "axis": None})


def _patterned(names, cfg, extra_disabled=(), base_entries=()) -> dict[str, Any]:
    """base_disable_all + ``names`` x (weight, input) with ``cfg`` (or the given entries) +
    default_disabled_quantizers + extra disables: the layout of the reference's pattern presets."""
    qc = list(_BASE_DISABLE_ALL) + list(base_entries)
    for n in names:
        qc += [{"quantizer_name": n + "weight_quantizer", "cfg": cfg}, {"quantizer_name": n + "input_quantizer", "cfg": cfg}]
    qc += _DEFAULT_DISABLED_QUANTIZERS
    qc += [{"quantizer_name": n, "enable": False} for n in extra_disabled]
    return {"quant_cfg": copy.deepcopy(qc), "algorithm": "max"}


_MLP_PATTERNS = ["*mlp*", "*.mixer.up_proj.", "*.mixer.down_proj.", "*block_sparse_moe*", "*.experts.*"]
NVFP4_MLP_ONLY_CFG: dict[str, Any] = _patterned(_MLP_PATTERNS, _NVFP4)
NVFP4_OMLP_ONLY_CFG: dict[str, Any] = _patterned(["*o_proj*"] + _MLP_PATTERNS[:4], _NVFP4)
NVFP4_EXPERTS_ONLY_CFG: dict[str, Any] = _patterned(["*block_sparse_moe*", "*.experts.*"], _NVFP4)
NVFP4_MLP_WEIGHT_ONLY_CFG: dict[str, Any] = {
    "quant_cfg": copy.deepcopy(
        _BASE_DISABLE_ALL
        + [{"quantizer_name": "*mlp*weight_quantizer", "cfg": _NVFP4_B32},
           {"quantizer_name": "*block_sparse_moe*weight_quantizer", "cfg": _NVFP4_B32}]
        + _DEFAULT_DISABLED_QUANTIZERS
    ),
    "algorithm": "max",
}
_MAMBA_MOE_AGGRESSIVE_OFF = ["*fc1_latent_proj*", "*fc2_latent_proj*", "*q_proj*", "*k_proj*", "*v_proj*",
                             "*o_proj*", "*self_attention.linear_qkv*", "*self_attention.linear_proj*"]
_MAMBA_MOE_CONSERVATIVE_OFF = _MAMBA_MOE_AGGRESSIVE_OFF + ["*mixer.in_proj*", "*mixer.out_proj*"]


def _mamba_moe(fmt, off) -> dict[str, Any]:
    c = _preset(fmt, fmt)
    c["quant_cfg"] += [{"quantizer_name": n, "enable": False} for n in off]
    return c


MAMBA_MOE_FP8_AGGRESSIVE_CFG: dict[str, Any] = _mamba_moe(_FP8_PT, _MAMBA_MOE_AGGRESSIVE_OFF)
MAMBA_MOE_FP8_CONSERVATIVE_CFG: dict[str, Any] = _mamba_moe(_FP8_PT, _MAMBA_MOE_CONSERVATIVE_OFF)
MAMBA_MOE_NVFP4_AGGRESSIVE_CFG: dict[str, Any] = _mamba_moe(_NVFP4, _MAMBA_MOE_AGGRESSIVE_OFF)
MAMBA_MOE_NVFP4_CONSERVATIVE_CFG: dict[str, Any] = _mamba_moe(_NVFP4, _MAMBA_MOE_CONSERVATIVE_OFF)
NVFP4_FOUR_OVER_SIX_CFG: dict[str, Any] = _preset(
    {"num_bits": (2, 1), "block_sizes": {-1: 16, "type": "static", "scale_bits": (4, 3), "four_over_six": 1}},
    _NVFP4,
    {"method": "mse", "fp8_scale_sweep": False, "start_multiplier": 1.0, "stop_multiplier": 1.5, "step_size": 0.5},
)

# Presets of algorithms / attributes outside this build's scope: defined so that code
# importing them keeps working; mtq.quantize raises NotImplementedError for smoothquant / svdquant /
# local_hessian (algorithm_config) and for rotated quantizers (TensorQuantizer).
INT8_SMOOTHQUANT_CFG: dict[str, Any] = _preset({"num_bits": 8, "axis": 0}, {"num_bits": 8, "axis": None},
                                               "smoothquant")
NVFP4_SVDQUANT_DEFAULT_CFG: dict[str, Any] = _preset(_NVFP4, _NVFP4, {"method": "svdquant", "lowrank": 32})
NVFP4_W4A4_WEIGHT_LOCAL_HESSIAN_CFG: dict[str, Any] = _preset(
    _NVFP4_STATIC, _NVFP4, {"method": "local_hessian", "fp8_scale_sweep": True}
)
NVFP4_KV_ROTATE_CFG: dict[str, Any] = {
    "quant_cfg": [
        {"quantizer_name": "*q_bmm_quantizer", "cfg": {"rotate": True}, "enable": False},
        {"quantizer_name": "*k_bmm_quantizer", "cfg": {**copy.deepcopy(_NVFP4), "rotate": True}},
        {"quantizer_name": "*v_bmm_quantizer", "cfg": copy.deepcopy(_NVFP4)},
    ],
    "algorithm": "max",
}

__all__ += [
    "W4A16_NVFP4_CFG",
    "W4A8_NVFP4_FP8_CFG",
    "NVFP4_MLP_ONLY_CFG",
    "NVFP4_OMLP_ONLY_CFG",
    "NVFP4_EXPERTS_ONLY_CFG",
    "NVFP4_MLP_WEIGHT_ONLY_CFG",
    "MAMBA_MOE_FP8_AGGRESSIVE_CFG",
    "MAMBA_MOE_FP8_CONSERVATIVE_CFG",
    "MAMBA_MOE_NVFP4_AGGRESSIVE_CFG",
    "MAMBA_MOE_NVFP4_CONSERVATIVE_CFG",
    "NVFP4_FOUR_OVER_SIX_CFG",
    "INT8_SMOOTHQUANT_CFG",
    "NVFP4_SVDQUANT_DEFAULT_CFG",
    "NVFP4_W4A4_WEIGHT_LOCAL_HESSIAN_CFG",
    "NVFP4_KV_ROTATE_CFG",
]
__all__ += [
    "FP8_2D_BLOCKWISE_WEIGHT_ONLY_CFG",
    "FP8_DEFAULT_CFG",
    "FP8_PER_CHANNEL_PER_TOKEN_CFG",
    "INT4_AWQ_CFG",
    "INT4_BLOCKWISE_WEIGHT_ONLY_CFG",
    "INT8_DEFAULT_CFG",
    "INT8_WEIGHT_ONLY_CFG",
    "MXFP4_DEFAULT_CFG",
    "MXFP4_MLP_WEIGHT_ONLY_CFG",
    "MXFP6_DEFAULT_CFG",
    "MXFP8_DEFAULT_CFG",
    "MXINT8_DEFAULT_CFG",
    "W4A8_MXFP4_FP8_CFG",
    "NVFP4_DEFAULT_CFG",
    "NVFP4_AWQ_LITE_CFG",
    "NVFP4_AWQ_CLIP_CFG",
    "NVFP4_AWQ_FULL_CFG",
    "NVFP4_W4A4_WEIGHT_MSE_FP8_SWEEP_CFG",
    "W4A8_AWQ_BETA_CFG",
    "FP8_KV_CFG",
    "NVFP4_KV_CFG",
    "FP8_AFFINE_KV_CFG",
    "NVFP4_AFFINE_KV_CFG",
    "NVFP4_FP8_MHA_CONFIG",
]

ForwardLoop = Callable[[Any], Any]
