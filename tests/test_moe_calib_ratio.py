"""``moe_calib_experts_ratio`` on a sparse sequential MoE block (experts as separate modules),
reference plugins/huggingface.py:623-750 + mode.py:240-247, run on the CPU path (INT8)."""

import pytest
import torch
import torch.nn as nn

import modelopt_amd.torch.quantization as mtq

H, E, N = 32, 8, 64


class Router(nn.Module):
    """transformers-5 TopKRouter shape: returns (logits, scores, indices)."""

    def __init__(self):
        super().__init__()
        self.weight = nn.Parameter(torch.randn(E, H) * 0.1)
        self.top_k, self.num_experts = 1, E

    def forward(self, x):
        logits = x @ self.weight.t()
        logits = logits + torch.arange(E, dtype=x.dtype) * -10.0  # rig: expert 0 wins at top-1
        scores, idx = torch.topk(logits.softmax(-1), self.top_k, dim=-1)
        return logits, scores, idx


class Expert(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(H, H)

    def forward(self, x):
        return self.fc(x)


class SparseMoe(nn.Module):
    def __init__(self):
        super().__init__()
        self.gate = Router()
        self.experts = nn.ModuleList([Expert() for _ in range(E)])

    def forward(self, x):
        _, scores, idx = self.gate(x)
        out = torch.zeros_like(x)
        for e in range(E):
            hit = (idx == e).any(-1)
            if hit.any():
                w = (scores * (idx == e)).sum(-1, keepdim=True)[hit]
                out[hit] += self.experts[e](x[hit]) * w
        return out


class Model(nn.Module):
    def __init__(self):
        super().__init__()
        self.moe = SparseMoe()

    def forward(self, x):
        return self.moe(x)


def _run(ratio, seen):
    torch.manual_seed(0)
    m = Model()
    hooks = [ex.fc.register_forward_pre_hook(lambda mod, a, i=i: seen.__setitem__(i, seen.get(i, 0) + a[0].shape[0]))
             for i, ex in enumerate(m.moe.experts)]
    cfg = {"quant_cfg": mtq.INT8_DEFAULT_CFG["quant_cfg"], "algorithm": {"method": "max"}}
    if ratio is not None:
        cfg["algorithm"]["moe_calib_experts_ratio"] = ratio
    x = torch.randn(N, H)
    mtq.quantize(m, cfg, lambda mm: mm(x))
    for h in hooks:
        h.remove()
    return m, x


def test_ratio_routes_calibration_tokens_to_all_experts():
    seen = {}
    m, x = _run(1.0, seen)
    assert type(m.moe).__name__.startswith("Quant")
    assert m.moe._moe_calib_experts_ratio == 1.0
    # the calibration forward ran once with top_k = E (every expert sees all N tokens) and once
    # with the original top_k = 1 (expert 0 sees all tokens)
    assert seen == {**{i: N for i in range(1, E)}, 0: 2 * N}
    assert m.moe.gate.top_k == 1
    for ex in m.moe.experts:
        assert ex.fc.input_quantizer.amax is not None
        assert torch.equal(ex.fc.input_quantizer.amax, x.abs().amax())


def test_ratio_half_counts_expert_tokens():
    seen = {}
    m, _ = _run(0.5, seen)
    assert hasattr(m.moe, "expert_token_count")
    # top_k raised to round(8 * 0.5) = 4 for the calibration-only pass: experts 0-3 get N each
    assert m.moe.expert_token_count.tolist() == [N] * 4 + [0] * 4


def test_without_ratio_experts_without_tokens_get_synced_amax():
    seen = {}
    m, x = _run(None, seen)
    assert seen == {0: N}
    a0 = m.moe.experts[0].fc.input_quantizer.amax
    for ex in m.moe.experts:  # layer_sync_moe_local_experts_amax: input amax max-synced
        assert torch.equal(ex.fc.input_quantizer.amax, a0)
        assert ex.fc.weight_quantizer.amax is not None


@pytest.mark.parametrize("bad", [0.0, 1.5, -1.0])
def test_ratio_validated(bad):
    with pytest.raises(Exception):
        mtq.config.MaxCalibConfig(moe_calib_experts_ratio=bad)
