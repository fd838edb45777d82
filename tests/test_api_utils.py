"""The reference's small public helpers around mtq.quantize, restated (CPU; INT8 runs on the
product's host kernels, the reference's "cpu" registration):

* ``find_quant_cfg_entry_by_path`` (config.py:245-276), ``LayerwiseConfig`` (:712-770);
* ``update_quant_cfg_with_kv_cache_quant`` (utils/core_utils.py:1049-1075);
* ``preserve_quantizer_attributes_context`` (conversion.py:507-567);
* ``temporarily_fold_weights`` (model_quant.py:740-806), ``compute_quantization_mse`` (:809-882).
"""

import copy

import pytest
import torch
import torch.nn as nn

import modelopt_amd.torch.quantization as mtq


def test_find_quant_cfg_entry_by_path_returns_last_exact_match():
    cfg = mtq.FP8_DEFAULT_CFG["quant_cfg"] + [{"quantizer_name": "*input_quantizer", "enable": False}]
    assert mtq.find_quant_cfg_entry_by_path(cfg, "*input_quantizer") == {"quantizer_name": "*input_quantizer",
                                                                        "enable": False}
    assert mtq.find_quant_cfg_entry_by_path(cfg, "*weight_quantizer")["cfg"]["num_bits"] == (4, 3)
    with pytest.raises(KeyError):
        mtq.find_quant_cfg_entry_by_path(cfg, "*q_proj.input_quantizer")  # no wildcard matching


def test_layerwise_config_fields():
    c = mtq.LayerwiseConfig(enable=True, checkpoint_dir="/tmp/x", save_every=3)
    assert c.enable and c.checkpoint_dir == "/tmp/x" and c.save_every == 3
    assert c.get_qdq_activations_from_prev_layer is False and c.calib_mutates_weights is True
    with pytest.raises(ValueError):
        mtq.LayerwiseConfig(save_every=0)


def test_update_quant_cfg_with_kv_cache_quant():
    base = copy.deepcopy(mtq.FP8_DEFAULT_CFG)
    out = mtq.update_quant_cfg_with_kv_cache_quant(base, mtq.FP8_KV_CFG["quant_cfg"])
    assert out["quant_cfg"][: len(base["quant_cfg"])] == base["quant_cfg"]
    assert out["quant_cfg"][-1] == mtq.FP8_KV_CFG["quant_cfg"][0]
    assert base == mtq.FP8_DEFAULT_CFG  # the input is not modified
    kv_only = mtq.update_quant_cfg_with_kv_cache_quant({"quant_cfg": None}, mtq.FP8_KV_CFG["quant_cfg"])
    assert kv_only["quant_cfg"][0] == {"quantizer_name": "*", "enable": False}
    assert kv_only["algorithm"] == "max"


def _int8_linear():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(32, 32), nn.ReLU(), nn.Linear(32, 16))
    data = [torch.randn(4, 32) for _ in range(3)]
    mtq.quantize(m, mtq.INT8_DEFAULT_CFG, lambda mm: [mm(d) for d in data])
    return m, data


def test_preserve_quantizer_attributes_context_restores_properties():
    m, _ = _int8_linear()
    q = m[0].input_quantizer
    before = q.get_modelopt_state(properties_only=True)
    with mtq.preserve_quantizer_attributes_context(m):
        mtq.set_quantizer_by_cfg(m, [{"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 4}}])
        q.disable()
        assert q.num_bits == 4 and not q.is_enabled
    assert q.num_bits == 8 and q.is_enabled
    assert q.get_modelopt_state(properties_only=True) == before


def test_temporarily_fold_weights_restores_weights():
    m, data = _int8_linear()
    w0 = m[0].weight.detach().clone()
    qdq = m[0].weight_quantizer(m[0].weight).detach().clone()
    with torch.no_grad():
        ref = m(data[0])
    with mtq.temporarily_fold_weights(m):
        assert torch.equal(m[0].weight.detach(), qdq)  # folded: the weight is its own qdq
        with torch.no_grad():
            inside = m(data[0])
    assert torch.equal(inside, ref)
    assert torch.equal(m[0].weight.detach(), w0)  # restored in place
    assert m[0].weight_quantizer.is_enabled


def test_compute_quantization_mse():
    m, data = _int8_linear()
    mse = mtq.compute_quantization_mse(m, lambda mm: [mm(d) for d in data], wildcards="*input_quantizer")
    assert set(mse) == {"0.input_quantizer", "2.input_quantizer"}
    # the first linear's input is the data itself
    q = m[0].input_quantizer
    want = sum(torch.mean((d - q(d)) ** 2).item() for d in data) / len(data)
    assert mse["0.input_quantizer"] == pytest.approx(want, rel=1e-12)
    m[2].input_quantizer.disable()
    assert "2.input_quantizer" not in mtq.compute_quantization_mse(m, lambda mm: mm(data[0]))
