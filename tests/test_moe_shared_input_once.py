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


class _EPExperts(torch.nn.Module):
    """A fused-experts module whose router may send a row to the sentinel E (expert parallelism:
    the expert lives on another rank): such rows reach no local F.linear."""

    def __init__(self, E=3, H=16, inter=24):
        super().__init__()
        self.num_experts = E
        g = torch.Generator().manual_seed(62)
        self.gate_up_proj = torch.nn.Parameter(torch.randn(E, 2 * inter, H, generator=g) * 0.2)
        self.down_proj = torch.nn.Parameter(torch.randn(E, H, inter, generator=g) * 0.2)

    def forward(self, hidden_states, top_k_index, top_k_weights):
        out = torch.zeros_like(hidden_states)
        for e in range(self.num_experts):
            tok, pos = torch.where(top_k_index == e)
            if tok.numel() == 0:
                continue
            gate, up = torch.nn.functional.linear(hidden_states[tok], self.gate_up_proj[e]).chunk(2, dim=-1)
            h = torch.nn.functional.linear(torch.nn.functional.silu(gate) * up, self.down_proj[e])
            out.index_add_(0, tok, h * top_k_weights[tok, pos, None])
        return out


def _ep_run(force_per_expert, monkeypatch):
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.plugins import huggingface as hf

    orig = hf._token_separable
    monkeypatch.setattr(hf, "_token_separable", (lambda q: False) if force_per_expert else orig)
    g = torch.Generator().manual_seed(63)
    hs = torch.randn(10, 16, generator=g)
    hs[3] *= 50.0  # the largest row goes to the sentinel only: it must not set the amax
    idx = torch.randint(0, 3, (10, 2), generator=g)
    idx[3] = 3
    idx[7, 1] = 3  # a row with one local and one remote expert
    w = torch.rand(10, 2, generator=g)

    class Wrap(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.experts = _EPExperts()

        def forward(self, x):
            return self.experts(x, idx, w)

    model = mtq.quantize(Wrap(), mtq.FP8_DEFAULT_CFG, lambda m: m(hs))
    with torch.no_grad():
        out = model(hs)
    monkeypatch.setattr(hf, "_token_separable", orig)
    return model.experts.gate_up_proj_input_quantizer.amax.float(), out, hs[(idx < 3).any(-1)]


def test_sentinel_rows_do_not_reach_the_shared_input_amax(monkeypatch):
    """Rows routed only to the sentinel are excluded from the once-per-forward input amax without
    a host sync (zeroed on the device): amax and outputs equal the per-expert calls'."""
    a1, o1, routed = _ep_run(False, monkeypatch)
    a0, o0, _ = _ep_run(True, monkeypatch)
    assert torch.equal(a1, routed.abs().amax().float())
    assert torch.equal(a1, a0)
    assert torch.isfinite(o1).all() and torch.equal(o1, o0)


def test_token_separable_nvfp4_needs_a_static_global_amax():
    """NVFP4 (dynamic block-16, E4M3 scales): the second-level scale uses the global amax, which
    without a static `_amax` is taken from the call's own input -- not token-separable then."""
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig
    from modelopt_amd.torch.quantization.plugins import huggingface as hf

    attrs = next(e["cfg"] for e in mtq.NVFP4_DEFAULT_CFG["quant_cfg"] if e["quantizer_name"] == "*input_quantizer")
    q = mtq.TensorQuantizer(QuantizerAttributeConfig(**attrs))
    assert q.block_sizes.get("scale_bits") == (4, 3)
    assert not hf._token_separable(q)
    q.amax = torch.tensor(3.0)
    assert hf._token_separable(q)


def test_installed_fused_experts_forward_reads_only_routed_rows(monkeypatch):
    """Pins the assumption behind the collect-only late path: the installed
    transformers fused-experts forward (MixtralExperts, eager) feeds its first projection of expert
    e exactly hidden_states[tokens routed to e] -- no dense product over all tokens -- so a shared
    input quantizer collected once on hidden_states sees what the per-expert calls would.  If an
    upstream release changes the loop (e.g. a dense matmul before the gather), this fails."""
    from transformers import MixtralConfig
    from transformers.models.mixtral.modeling_mixtral import MixtralExperts

    cfg = MixtralConfig(hidden_size=16, intermediate_size=24, num_local_experts=4, num_experts_per_tok=2)
    cfg._experts_implementation = "eager"
    ex = MixtralExperts(cfg)
    g = torch.Generator().manual_seed(64)
    with torch.no_grad():
        ex.gate_up_proj.normal_(0, 0.2, generator=g)
        ex.down_proj.normal_(0, 0.2, generator=g)
    hs = torch.randn(12, 16, generator=g)
    idx = torch.stack([torch.randperm(4, generator=g)[:2] for _ in range(12)])
    idx[5] = torch.tensor([1, 3])  # expert 0 and 2 skipped by this row
    wts = torch.rand(12, 2, generator=g)
    seen = []
    orig = torch.nn.functional.linear

    def spy(x, w, b=None):
        seen.append((x, w))
        return orig(x, w, b)

    monkeypatch.setattr(torch.nn.functional, "linear", spy)
    with torch.no_grad():
        ex(hs, idx, wts)
    first = [(x, w) for x, w in seen if w.shape == ex.gate_up_proj.shape[1:]]
    assert sum(x.shape[0] for x, _ in first) == idx.numel()  # every (token, k) pair once
    for x, w in first:
        e = (w.storage_offset() - ex.gate_up_proj.storage_offset()) // ex.gate_up_proj.stride(0)
        tok = (idx == e).any(-1).nonzero().flatten()
        # each row of the gather is one routed token's hidden state (in the loop's own order)
        src = [int((hs == r).all(-1).nonzero().flatten()[0]) for r in x]
        assert sorted(src) == tok.tolist(), e
        assert torch.equal(x, hs[src]), e
