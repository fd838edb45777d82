"""KV-cache / attention-BMM quantizers (reference plugins/huggingface.py:78-460 ``_QuantAttention``)
on the GPU vs the reference's outputs (tests/golden/kv.*, made by running the reference on the
CPU: tiny Llama with FP8 W/A plus FP8 K/V, constant-amax FP8 K/V, FP8 Q/K/V, INT8 K/V)."""

import copy
import json
from pathlib import Path

import pytest
import torch
from safetensors.torch import load_file

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"
META = json.loads((G / "kv.json").read_text())


@pytest.fixture(scope="module")
def gold():
    return load_file(str(G / "kv.safetensors"))


def _tiny():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=32, max_position_embeddings=64,
                      architectures=["LlamaForCausalLM"])
    torch.manual_seed(80)
    return LlamaForCausalLM(cfg).eval()


def _cfg(mtq, name):
    cfg = copy.deepcopy(mtq.FP8_DEFAULT_CFG)
    fp8 = {"num_bits": (4, 3), "axis": None}
    cfg["quant_cfg"] = cfg["quant_cfg"] + {
        "fp8_kv": [{"quantizer_name": "*[kv]_bmm_quantizer", "cfg": dict(fp8)}],
        "fp8_kv_cast": [{"quantizer_name": "*[kv]_bmm_quantizer", "cfg": dict(fp8, use_constant_amax=True)}],
        "qkv_fp8": [{"quantizer_name": "*[qkv]_bmm_quantizer", "cfg": dict(fp8)}],
        "int8_kv": [{"quantizer_name": "*[kv]_bmm_quantizer", "cfg": {"num_bits": 8, "axis": None}}],
    }[name]
    return cfg


@pytest.mark.parametrize("name", sorted(META))
def test_kv_calibration_matches_reference(gpu, gold, name):
    import modelopt_amd.torch.quantization as mtq

    m = _tiny().to(gpu)
    ids = gold["calib_ids"].to(gpu)
    mtq.quantize(m, _cfg(mtq, name), lambda mm: [mm(b) for b in ids])
    enabled = [n for n, q in m.named_modules() if isinstance(q, mtq.TensorQuantizer) and q.is_enabled]
    assert enabled == META[name]["enabled"]
    n_bmm = 0
    for k, v in gold.items():
        if not k.startswith(f"{name}.amax."):
            continue
        qn = k[len(f"{name}.amax."):]
        q = m.get_submodule(qn)
        if qn.endswith("weight_quantizer"):
            assert torch.equal(q._amax.cpu(), v), qn
        else:  # activations: GEMM outputs differ in the last bits between CPU and GPU
            torch.testing.assert_close(q._amax.cpu(), v, rtol=2e-5, atol=0)
        n_bmm += "bmm" in qn
    assert n_bmm == {"fp8_kv": 4, "fp8_kv_cast": 0, "qkv_fp8": 6, "int8_kv": 4}[name]
    if name == "fp8_kv_cast":
        assert all(m.get_submodule(n)._use_constant_amax for n in enabled if "bmm" in n)
    with torch.no_grad():
        logits = m(gold["test_ids"].to(gpu)).logits
    torch.testing.assert_close(logits.cpu(), gold[f"{name}.logits"], rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("name", ["fp8_kv", "fp8_kv_cast"])
def test_kv_export_matches_reference(gpu, gold, name, tmp_path):
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.export import export_hf_checkpoint

    m = _tiny().to(gpu)
    ids = gold["calib_ids"].to(gpu)
    mtq.quantize(m, _cfg(mtq, name), lambda mm: [mm(b) for b in ids])
    state = {k[len(name) + 7:]: v for k, v in gold.items() if k.startswith(name + ".state.")}
    missing, unexpected = m.load_state_dict(state, strict=False)
    assert not unexpected, unexpected
    export_hf_checkpoint(m, export_dir=str(tmp_path))
    got = load_file(str(tmp_path / "model.safetensors"))
    want = {k[len(name) + 8:]: v for k, v in gold.items() if k.startswith(name + ".export.")}
    assert set(got) == set(want), sorted(set(got) ^ set(want))[:10]
    for k, v in want.items():
        g = got[k]
        assert g.dtype == v.dtype and g.shape == v.shape, k
        assert torch.equal(g.view(torch.uint8) if g.element_size() == 1 else g,
                           v.view(torch.uint8) if v.element_size() == 1 else v), k
    hq = json.loads((tmp_path / "hf_quant_config.json").read_text())
    hq["producer"]["version"] = None
    assert hq == META[name]["hf_quant_config"]
    cq = json.loads((tmp_path / "config.json").read_text())["quantization_config"]
    cq["producer"]["version"] = None
    assert cq == META[name]["quantization_config"]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_per_tensor_qdq_reads_strided_states_in_place(gpu, dtype):
    """K/V states arrive as transposed [B, H, S, D] views: the per-tensor FP8 / INT8 qdq and the
    amax reduction run on them in storage order, bit-identical to the contiguous path."""
    from modelopt_amd.torch.quantization.tensor_quant import fp8_fake_quant, quantize_op
    from modelopt_amd.torch.quantization.utils import reduce_amax

    x = (torch.randn(2, 37, 8, 64, device=gpu) * 3).to(dtype).transpose(1, 2)  # [B, H, S, D] view
    assert not x.is_contiguous()
    a = reduce_amax(x)
    assert torch.equal(a, reduce_amax(x.contiguous()))
    amax = a.float()
    y = fp8_fake_quant(x, amax)
    assert y.stride() == x.stride()
    assert torch.equal(y.contiguous(), fp8_fake_quant(x.contiguous(), amax))
    assert torch.equal(y.cpu().float().contiguous(), R.fp8_eager(x.cpu().contiguous(), amax.cpu()).float())
    yi = quantize_op(x, amax, 8, 0, False, False)
    assert yi.stride() == x.stride()
    assert torch.equal(yi.contiguous(), quantize_op(x.contiguous(), amax, 8, 0, False, False))


# p_bmm_quantizer (softmax-P qdq): tests/test_gpu_attention.py -- the causal path runs the fused
# MFMA flash attention as the reference dispatches it (plugins/huggingface.py:236-251).
