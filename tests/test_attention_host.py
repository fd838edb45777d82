"""Host logic of the fused attention path (no GPU): argument checks and error behaviour mirror
the reference's attention() / validate_triton_attention_envelope (triton_fa.py:1221-1390,
hf_triton_attention.py:96-151), the P-qdq scale conventions, and the plugin's format mapping
(plugins/huggingface.py:125-143)."""

import pytest
import torch


def test_scale_conventions():
    from modelopt_amd.torch.kernels.common.attention.flash_attention import _p_qdq_scale

    assert _p_qdq_scale("fp8", 1.0) == 1.0 / 448.0
    assert _p_qdq_scale("nvfp4", 0.5) == 0.5 / (6.0 * 448.0)
    assert _p_qdq_scale(None, 3.0) == 1.0
    for bad in (0.0, -1.0, float("inf"), float("nan")):
        with pytest.raises(ValueError):
            _p_qdq_scale("fp8", bad)


def test_attention_argument_errors():
    from modelopt_amd.torch.kernels.common.attention import attention

    q = torch.zeros(4, 2, 64, dtype=torch.bfloat16)
    meta = (torch.zeros(1, dtype=torch.int32), torch.tensor([4], dtype=torch.int32), 4)
    with pytest.raises(ValueError):
        attention(q, q, q, *meta, p_qdq="int8")
    with pytest.raises(NotImplementedError):
        attention(q, q, q, *meta, sparsity_n=2)
    with pytest.raises(NotImplementedError):
        attention(q, q, q, *meta, skip_softmax_threshold=0.1)
    with pytest.raises(RuntimeError, match="ROCm"):  # no CPU path, no fallback
        attention(q, q, q, *meta, p_qdq="fp8")


def test_envelope_matches_reference_rules():
    from modelopt_amd.torch.kernels.common.attention import validate_attention_envelope

    class M(torch.nn.Module):
        is_causal = True

    q = torch.zeros(1, 2, 8, 64)
    validate_attention_envelope(M(), q, q, None)
    with pytest.raises(NotImplementedError, match="sliding-window"):
        validate_attention_envelope(M(), q, q, None, sliding_window=4)
    with pytest.raises(NotImplementedError, match="non-causal"):
        validate_attention_envelope(M(), q, q, None, is_causal=False)
    with pytest.raises(NotImplementedError, match="longer KV cache"):
        validate_attention_envelope(M(), q, torch.zeros(1, 2, 12, 64), None)
    left = torch.ones(1, 8)
    left[0, 0] = 0
    with pytest.raises(NotImplementedError, match="left-padded"):
        validate_attention_envelope(M(), q, q, left)
    holed = torch.ones(1, 8)
    holed[0, 3] = 0
    with pytest.raises(NotImplementedError, match="non-contiguously"):
        validate_attention_envelope(M(), q, q, holed)
    right = torch.ones(1, 8)
    right[0, 6:] = 0
    validate_attention_envelope(M(), q, q, right)


def test_plugin_p_qdq_mode_mapping():
    from modelopt_amd.torch.quantization.nn import TensorQuantizer
    from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig
    from modelopt_amd.torch.quantization.plugins.huggingface import _QuantAttention

    class Holder:
        _p_qdq_mode = _QuantAttention._p_qdq_mode

    def mode(cfg):
        h = Holder()
        h.p_bmm_quantizer = TensorQuantizer(QuantizerAttributeConfig(**cfg))
        return h._p_qdq_mode()

    assert mode({"num_bits": (4, 3), "axis": None}) == "fp8"
    nv = {"num_bits": (2, 1), "block_sizes": {-1: 16, "type": "dynamic", "scale_bits": (4, 3)}, "axis": None}
    assert mode(nv) == "nvfp4"
    assert mode(dict(nv, block_sizes={-1: 32, "type": "dynamic", "scale_bits": (4, 3)})) is None
    assert mode({"num_bits": 8, "axis": None}) is None
    assert mode({"num_bits": (4, 3), "axis": None, "enable": False}) is None
