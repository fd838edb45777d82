"""Fused-experts MoE (plugins/huggingface.py _QuantFusedExperts; reference :976-1115): the shared
first-projection input quantizer applied once to the layer's hidden states must give exactly what
the per-expert application over each expert's token gather gives (the reference's order): same
amax after calibration, same logits after quantization.  CPU path (tiny Mixtral, FP8_DEFAULT_CFG
and an NVFP4 dynamic-block input), compared with the per-expert calls forced."""

import pytest
import torch


def _tiny_mixtral():
    from transformers import MixtralConfig, MixtralForCausalLM

    cfg = MixtralConfig(hidden_size=32, intermediate_size=48, num_hidden_layers=2, num_attention_heads=4,
                        num_key_value_heads=2, vocab_size=32, max_position_embeddings=64, num_local_experts=4,
                        num_experts_per_tok=2)
    torch.manual_seed(60)
    return MixtralForCausalLM(cfg).eval()


def _run(cfg_name, monkeypatch, force_per_expert):
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.plugins import huggingface as hf

    calls = {"n": 0}
    orig = hf._token_separable

    def spy(q):
        r = False if force_per_expert else orig(q)
        calls["n"] += int(r)
        return r

    monkeypatch.setattr(hf, "_token_separable", spy)
    g = torch.Generator().manual_seed(61)
    ids = torch.randint(0, 32, (3, 2, 16), generator=g)
    model = mtq.quantize(_tiny_mixtral(), getattr(mtq, cfg_name), lambda m: [m(b) for b in ids])
    with torch.no_grad():
        logits = model(torch.randint(0, 32, (2, 16), generator=g)).logits
    amax = {n: m.amax.clone() for n, m in model.named_modules()
            if isinstance(m, mtq.TensorQuantizer) and m.is_enabled and getattr(m, "_amax", None) is not None}
    return amax, logits, calls["n"]


@pytest.mark.parametrize("cfg_name", ["FP8_DEFAULT_CFG", "INT8_DEFAULT_CFG"])
def test_shared_input_once_equals_per_expert(cfg_name, monkeypatch):
    a1, l1, n1 = _run(cfg_name, monkeypatch, force_per_expert=False)
    a0, l0, _ = _run(cfg_name, monkeypatch, force_per_expert=True)
    assert n1 > 0  # the once-per-forward path was taken
    assert a1.keys() == a0.keys() and any("gate_up_proj_input_quantizer" in k for k in a1)
    for k in a1:
        assert torch.equal(a1[k], a0[k]), k
    assert torch.equal(l1, l0)
