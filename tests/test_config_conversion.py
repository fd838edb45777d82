"""Host logic on CPU: presets equal the reference's, config validation, module conversion and
ordered wildcard configuration (reference tests: tests/unit/torch/quantization/test_config*.py,
test_quantize_cpu.py)."""

import json
from pathlib import Path

import pytest
import torch
import torch.nn as nn

import modelopt_amd.torch.quantization as mtq
from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig, normalize_quant_cfg_list
from modelopt_amd.torch.quantization.nn import TensorQuantizer

G = Path(__file__).resolve().parent / "golden"


def _dec(o):
    if isinstance(o, dict):
        if set(o) == {"__tuple__"}:
            return tuple(_dec(v) for v in o["__tuple__"])
        return {(int(k[7:]) if isinstance(k, str) and k.startswith("__int__") else k): _dec(v) for k, v in o.items()}
    if isinstance(o, list):
        return [_dec(v) for v in o]
    return o


@pytest.mark.parametrize("name", sorted(json.loads((G / "presets.json").read_text())))
def test_presets_match_reference(name):
    ref = _dec(json.loads((G / "presets.json").read_text())[name])
    assert getattr(mtq, name) == ref


def test_attribute_config_validation():
    QuantizerAttributeConfig(num_bits=(4, 3))
    QuantizerAttributeConfig(num_bits="e4m3")
    with pytest.raises(ValueError):
        QuantizerAttributeConfig(num_bits=(3, 2))  # E3M2 needs dynamic blocks
    QuantizerAttributeConfig(num_bits=(3, 2), block_sizes={-1: 32, "type": "dynamic", "scale_bits": (8, 0)})
    with pytest.raises(ValueError):
        QuantizerAttributeConfig(enable=True)
    with pytest.raises(ValueError):
        QuantizerAttributeConfig(axis=0, block_sizes={-1: 128})
    assert QuantizerAttributeConfig().narrow_range is False


def test_normalize_list_and_legacy_dict():
    lst = normalize_quant_cfg_list([{"quantizer_name": "*", "enable": False},
                                    {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 8}}])
    assert lst[0]["cfg"] is None and lst[0]["enable"] is False
    assert lst[1]["enable"] is True and lst[1]["cfg"] == {"num_bits": 8}
    legacy = normalize_quant_cfg_list({"*weight_quantizer": {"num_bits": 4, "enable": True}, "default": {"enable": False}})
    assert legacy[0]["quantizer_name"] == "*weight_quantizer" and legacy[0]["enable"] is True
    assert legacy[1]["quantizer_name"] == "*" and legacy[1]["enable"] is False
    with pytest.raises(ValueError):
        normalize_quant_cfg_list([{"quantizer_name": "*"}])


class Tiny(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(16, 32)
        self.lm_head = nn.Linear(32, 8)
        self.emb = nn.Embedding(4, 16)

    def forward(self, x):
        return self.lm_head(torch.relu(self.fc1(x)))


def test_convert_and_ordered_cfg():
    m = Tiny()
    w = m.fc1.weight
    mtq.conversion.replace_quant_module(m)
    assert type(m.fc1).__name__ == "QuantLinear" and isinstance(m.fc1, nn.Linear)
    assert m.fc1.weight is w  # parameters untouched
    mtq.set_quantizer_by_cfg(m, mtq.FP8_DEFAULT_CFG["quant_cfg"])
    assert m.fc1.weight_quantizer.is_enabled and m.fc1.weight_quantizer.num_bits == (4, 3)
    assert m.fc1.input_quantizer.is_enabled
    assert not m.lm_head.weight_quantizer.is_enabled  # *lm_head* disabled
    assert not m.fc1.output_quantizer.is_enabled
    # full replacement: later cfg resets unspecified attributes to defaults
    mtq.set_quantizer_by_cfg(m, [{"quantizer_name": "*fc1.weight_quantizer", "cfg": {"num_bits": 4, "axis": 0}}])
    q = m.fc1.weight_quantizer
    assert q.num_bits == 4 and q.axis == 0 and q.block_sizes is None and q.is_enabled
    # enable-only entry toggles without touching attributes
    mtq.set_quantizer_by_cfg(m, [{"quantizer_name": "*fc1.weight_quantizer", "enable": False}])
    assert not q.is_enabled and q.num_bits == 4
    # sequential quantizer via list cfg
    mtq.set_quantizer_by_cfg(m, [{"quantizer_name": "*fc1.weight_quantizer",
                                  "cfg": [{"num_bits": 4, "block_sizes": {-1: 8}}, {"num_bits": (4, 3)}]}])
    assert isinstance(m.fc1.weight_quantizer, mtq.SequentialQuantizer) and len(m.fc1.weight_quantizer) == 2


def test_export_restores_module():
    m = Tiny()
    mtq.conversion.replace_quant_module(m)
    m.fc1.export()
    assert type(m.fc1) is nn.Linear and not hasattr(m.fc1, "weight_quantizer")


def test_modelopt_state_roundtrip():
    q = TensorQuantizer(QuantizerAttributeConfig(num_bits=4, block_sizes={-1: 128, "type": "static"}))
    q.amax = torch.ones(3, 1)
    st = q.get_modelopt_state()
    assert st["_num_bits"] == 4 and st["_pytorch_state_metadata"]["buffers"]["_amax"]["shape"] == torch.Size([3, 1])
    q2 = TensorQuantizer()
    q2.set_from_modelopt_state(st)
    assert q2.num_bits == 4 and q2._amax.shape == (3, 1)


def test_block_sizes_to_axis_and_repr():
    q = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, block_sizes={-1: None}))
    q._block_sizes_to_axis(torch.empty(4, 5))
    assert q.block_sizes is None and q.axis == (0,)
    assert "8 bit" in repr(TensorQuantizer())


def test_backend_registry():
    calls = []
    mtq.register_quant_backend("echo", lambda x, tq: calls.append(1) or x * 2)
    q = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, backend="echo"))
    q.amax = torch.tensor(1.0)
    out = q(torch.ones(3))
    assert torch.equal(out, torch.full((3,), 2.0)) and calls == [1]
    mtq.unregister_quant_backend("echo")


def _tiny_mixtral():
    from transformers import MixtralConfig, MixtralForCausalLM

    cfg = MixtralConfig(hidden_size=32, intermediate_size=48, num_hidden_layers=2, num_attention_heads=4,
                        num_key_value_heads=2, vocab_size=32, max_position_embeddings=64,
                        num_local_experts=4, num_experts_per_tok=2)
    torch.manual_seed(60)
    return MixtralForCausalLM(cfg).eval()


def test_fused_experts_conversion_matches_reference():
    """C5 structure: the fused-experts plugin registers on the fly and yields the reference's
    quantizer set under FP8_DEFAULT_CFG (tests/golden/mixtral_fp8.json), including the attention
    q/k/v/p bmm quantizers (registered on the fly, disabled under this config)."""
    ref = json.loads((G / "mixtral_fp8.json").read_text())["quantizers"]
    want_enabled = {n for n, e in ref if e}
    want_all = {n for n, _ in ref}
    m = _tiny_mixtral()
    m.config._experts_implementation = "grouped_mm"
    mtq.conversion.replace_quant_module(m)
    assert m.config._experts_implementation == "eager"  # grouped_mm would bypass F.linear
    mtq.set_quantizer_by_cfg(m, mtq.FP8_DEFAULT_CFG["quant_cfg"])
    got = {n: q.is_enabled for n, q in m.named_modules() if isinstance(q, TensorQuantizer)}
    assert set(got) == want_all
    assert {n for n, e in got.items() if e} == want_enabled
    ex = m.model.layers[0].mlp.experts
    assert type(ex).__name__ == "QuantMixtralExperts"
    pairs = list(ex.iter_weights_for_calibration())
    assert len(pairs) == 8 and pairs[1][0].data_ptr() == ex.gate_up_proj[1].data_ptr()
    assert pairs[1][1] is ex.gate_up_proj_weight_quantizers[1]
    assert ex._get_expert_idx_from_first_proj(ex.gate_up_proj[3]) == 3


def test_max_calibrator_skips_same_view():
    from modelopt_amd.torch.quantization.calib import max as max_mod
    from modelopt_amd.torch.quantization.calib.max import MaxCalibrator

    p = nn.Parameter(torch.randn(4, 8, 16))
    c = MaxCalibrator()
    c._acc = torch.zeros(1)
    c._last = None
    base, key = c._view_key(p[2])
    import weakref

    c._last = (weakref.ref(base), key, p[2]._version, max_mod._EPOCH)
    assert c._same_as_last(p[2])  # a fresh view of the same slice
    assert not c._same_as_last(p[1])
    max_mod.new_collect_epoch()
    assert not c._same_as_last(p[2])  # a new collection pass forgets the key
    c._last = (weakref.ref(base), key, p[2]._version, max_mod._EPOCH)
    with torch.no_grad():
        p.mul_(2)
    assert not c._same_as_last(p[2])  # version bumped


@pytest.mark.parametrize("name", ["INT8_SMOOTHQUANT_CFG", "NVFP4_SVDQUANT_DEFAULT_CFG",
                                  "NVFP4_W4A4_WEIGHT_LOCAL_HESSIAN_CFG"])
def test_out_of_scope_presets_raise(name):
    """Presets of algorithms outside the MI355X path exist (import compatibility) and raise
    NotImplementedError when used, before any calibration work."""
    import torch
    import torch.nn as nn

    with pytest.raises(NotImplementedError):
        mtq.quantize(nn.Linear(16, 16), getattr(mtq, name), lambda m: m(torch.randn(2, 16)))


def test_rotated_kv_preset_raises():
    from modelopt_amd.torch.quantization.nn.modules.tensor_quantizer import TensorQuantizer

    with pytest.raises(NotImplementedError):
        TensorQuantizer(QuantizerAttributeConfig(**mtq.NVFP4_KV_ROTATE_CFG["quant_cfg"][1]["cfg"]))
