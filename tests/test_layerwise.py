"""Layerwise calibration machinery (skip / run / capture) on CPU: every decoder layer must be
handed exactly the hidden states a whole-model forward gives it (reference semantics with
get_qdq_activations_from_prev_layer=False), and checkpoint/resume must continue where it stopped."""

import pytest
import torch

from modelopt_amd.torch.quantization.layerwise import LayerActivationCollector, layerwise_calibrate


def _tiny_llama(layers=4):
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=32, intermediate_size=64, num_hidden_layers=layers, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=50, max_position_embeddings=64)
    torch.manual_seed(0)
    return LlamaForCausalLM(cfg).eval()


def _reference_inputs(model, batches, sub=None):
    """Inputs each decoder layer (or its submodule ``sub``, e.g. the attention output projection)
    receives in a whole-model forward."""
    seen = {i: [] for i in range(len(model.model.layers))}
    mods = [layer.get_submodule(sub) if sub else layer for layer in model.model.layers]
    hooks = [m.register_forward_pre_hook(lambda m, a, k, i=i: seen[i].append(a[0].clone() if a else k["hidden_states"].clone()), with_kwargs=True)
             for i, m in enumerate(mods)]
    with torch.no_grad():
        for b in batches:
            model(b)
    for h in hooks:
        h.remove()
    return seen


def test_decoder_layers_discovered():
    m = _tiny_llama()
    assert LayerActivationCollector.get_decoder_layers(m) is m.model.layers


@pytest.mark.parametrize("use_cache", [True, False])
def test_layerwise_inputs_match_whole_model(use_cache):
    m = _tiny_llama()
    m.config.use_cache = use_cache
    g = torch.Generator().manual_seed(1)
    batches = [torch.randint(0, 50, (2, 12), generator=g) for _ in range(3)]
    want = _reference_inputs(m, batches)
    want_o = _reference_inputs(m, batches, "self_attn.o_proj")
    got, got_o = {}, {}

    def calib(layer, loop):
        idx = list(m.model.layers).index(layer)
        got[idx], got_o[idx] = [], []
        h = layer.register_forward_pre_hook(lambda mod, a, k: got[idx].append(a[0].clone() if a else k["hidden_states"].clone()), with_kwargs=True)
        h2 = layer.self_attn.o_proj.register_forward_pre_hook(lambda mod, a: got_o[idx].append(a[0].clone()))
        loop(layer)
        loop(layer)  # a second replay (e.g. AWQ's cache + search passes) must see the same thing
        h.remove()
        h2.remove()

    layerwise_calibrate(m, lambda mm: [mm(b) for b in batches], calib)
    assert sorted(got) == list(range(4))
    for i in range(4):
        assert len(got[i]) == 6 and len(got_o[i]) == 6
        for a, b in zip(got[i], want[i] + want[i]):
            torch.testing.assert_close(a, b, rtol=0, atol=0)
        for a, b in zip(got_o[i], want_o[i] + want_o[i]):  # attention saw an empty KV cache
            torch.testing.assert_close(a, b, rtol=0, atol=0)
    # unpatched afterwards: the model runs normally
    assert "forward" not in m.__dict__ and all("forward" not in l.__dict__ for l in m.model.layers)
    with torch.no_grad():
        assert m(batches[0]).logits.shape == (2, 12, 50)


def test_layerwise_checkpoint_resume(tmp_path):
    m = _tiny_llama()
    g = torch.Generator().manual_seed(2)
    batches = [torch.randint(0, 50, (2, 8), generator=g) for _ in range(2)]
    calls = []

    class Stop(Exception):
        pass

    def calib_fail_at_2(layer, loop):
        idx = list(m.model.layers).index(layer)
        if idx == 2:
            raise Stop()
        calls.append(idx)
        loop(layer)

    with pytest.raises(Stop):
        layerwise_calibrate(m, lambda mm: [mm(b) for b in batches], calib_fail_at_2, checkpoint_dir=str(tmp_path))
    assert calls == [0, 1]
    want = _reference_inputs(m, batches)
    got = {}

    def calib(layer, loop):
        idx = list(m.model.layers).index(layer)
        got[idx] = []
        h = layer.register_forward_pre_hook(lambda mod, a, k: got[idx].append(a[0].clone() if a else k["hidden_states"].clone()), with_kwargs=True)
        loop(layer)
        h.remove()

    layerwise_calibrate(m, lambda mm: [mm(b) for b in batches], calib, checkpoint_dir=str(tmp_path))
    assert sorted(got) == [2, 3]  # resumed at the first unfinished layer
    for i in (2, 3):
        for a, b in zip(got[i], want[i]):
            torch.testing.assert_close(a, b, rtol=0, atol=0)
