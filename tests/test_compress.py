"""mtq.compress on the CPU path for the formats whose packing is a plain tensor expression
(INT8, INT4): packed bytes, scales, dequantised weights and logits bit-exact vs the reference's
own compress (tests/golden/compress.*); save / restore of a compressed model."""

import io

import pytest
import torch

from compress_cases import META, build, check_compressed


@pytest.mark.parametrize("case", ["int8", "int4"])
def test_compress_cpu_matches_reference(case):
    import modelopt_amd.torch.quantization as mtq

    m, t = build(case, "cpu")
    mtq.compress(m)
    assert mtq.is_real_quantized(m)
    assert not check_compressed(case, m, t)
    with torch.no_grad():
        logits = m(t["test_ids"]).logits.float()
    assert torch.equal(logits, t[f"{case}.logits"])


def test_compress_config_patterns():
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.qtensor import QTensorWrapper

    m, _ = build("int8", "cpu")
    mtq.compress(m, {"*mlp*": False, "default": True})
    for n, mod in m.named_modules():
        if n.endswith(("q_proj", "k_proj", "v_proj", "o_proj")):
            assert isinstance(mod.weight, QTensorWrapper), n
        if n.endswith(("gate_proj", "up_proj", "down_proj")):
            assert not isinstance(mod.weight, QTensorWrapper), n
            assert mod.weight_quantizer.fake_quant


def test_compressed_save_restore_roundtrip():
    import modelopt_amd.torch.opt as mto
    import modelopt_amd.torch.quantization as mtq
    from compress_cases import tiny_llama_bf16

    m, t = build("int4", "cpu")
    mtq.compress(m)
    buf = io.BytesIO()
    mto.save(m, buf)
    buf.seek(0)
    fresh = tiny_llama_bf16()
    mto.restore(fresh, buf)
    with torch.no_grad():
        assert torch.equal(fresh(t["test_ids"]).logits.float(), t["int4.logits"])
    assert not check_compressed("int4", fresh, t)
