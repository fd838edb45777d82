"""Fused-experts MoE with an NVFP4 (dynamic block-16, E4M3 scales) shared input quantizer
(plugins/huggingface.py `_token_separable`; reference plugins/huggingface.py:976-1115,
which applies the input quantizer to each expert's token gather).

NVFP4's second-level scale comes from the global amax.  With a calibrated (static) global amax the
quantizer treats every token on its own, so one application to all routed tokens equals the
per-expert calls; without one the global amax is the amax of whatever the call sees, so the
once-per-forward path must not be taken -- the per-expert gathers each get their own global amax,
as in the reference."""

import pytest
import torch


def _tiny_mixtral():
    from transformers import MixtralConfig, MixtralForCausalLM

    cfg = MixtralConfig(hidden_size=64, intermediate_size=96, num_hidden_layers=2, num_attention_heads=4,
                        num_key_value_heads=2, vocab_size=32, max_position_embeddings=64, num_local_experts=4,
                        num_experts_per_tok=2)
    torch.manual_seed(70)
    return MixtralForCausalLM(cfg).eval()


def _run(gpu, monkeypatch, calibrate: bool, force_per_expert: bool):
    import copy

    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.plugins import huggingface as hf

    seen = {"once": 0, "asked": 0}
    orig = hf._token_separable

    def spy(q):
        r = False if force_per_expert else orig(q)
        seen["asked"] += 1
        seen["once"] += int(r)
        return r

    monkeypatch.setattr(hf, "_token_separable", spy)
    cfg = copy.deepcopy(mtq.NVFP4_DEFAULT_CFG)
    if not calibrate:
        cfg["algorithm"] = None
    g = torch.Generator().manual_seed(71)
    ids = torch.randint(0, 32, (3, 2, 16), generator=g).to(gpu)
    model = _tiny_mixtral().to(gpu)
    model = mtq.quantize(model, cfg, (lambda m: [m(b) for b in ids]) if calibrate else None)
    with torch.no_grad():
        logits = model(torch.randint(0, 32, (2, 16), generator=g).to(gpu)).logits
    amax = {n: m.amax.clone() for n, m in model.named_modules()
            if isinstance(m, mtq.TensorQuantizer) and m.is_enabled and getattr(m, "_amax", None) is not None}
    monkeypatch.setattr(hf, "_token_separable", orig)
    return amax, logits, seen


@pytest.mark.gpu
def test_nvfp4_calibrated_input_once_equals_per_expert(gpu, monkeypatch):
    a1, l1, s1 = _run(gpu, monkeypatch, calibrate=True, force_per_expert=False)
    a0, l0, _ = _run(gpu, monkeypatch, calibrate=True, force_per_expert=True)
    assert s1["once"] > 0  # static global amax: the once-per-forward path is taken
    assert a1.keys() == a0.keys() and any("gate_up_proj_input_quantizer" in k for k in a1)
    for k in a1:
        assert torch.equal(a1[k], a0[k]), k
    assert torch.equal(l1, l0)


@pytest.mark.gpu
def test_nvfp4_dynamic_global_amax_keeps_per_expert_calls(gpu, monkeypatch):
    a1, l1, s1 = _run(gpu, monkeypatch, calibrate=False, force_per_expert=False)
    a0, l0, _ = _run(gpu, monkeypatch, calibrate=False, force_per_expert=True)
    assert s1["asked"] > 0 and s1["once"] == 0  # no static global amax: per-expert gathers
    assert torch.equal(l1, l0)
