"""End-to-end mtq.quantize on the GPU against the reference's CPU results (golden fixtures).

C1 (nn.Linear(1024,1024) INT8_DEFAULT_CFG), the C2 model class (tiny LlamaForCausalLM,
FP8_DEFAULT_CFG) and the C3 algorithm (awq_lite on a small MLP).  Weight-side amax is bit-exact
(same data, exact max); activation amax and outputs go through GEMMs whose summation order differs
between the reference's CPU run and hipBLASLt, so they are compared with a tolerance stated per test.
"""

from pathlib import Path

import json

import pytest
import torch
import torch.nn as nn
from safetensors.torch import load_file

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"


def test_c1_linear_int8(gpu):
    import modelopt_amd.torch.quantization as mtq

    t = load_file(str(G / "mtq_linear.safetensors"))
    m = nn.Linear(1024, 1024).to(gpu)
    m.load_state_dict({"weight": t["weight"], "bias": t["bias"]})
    calib = [t[f"calib{i}"].to(gpu) for i in range(4)]

    def loop(model):
        for c in calib:
            model(c)

    mtq.quantize(m, mtq.INT8_DEFAULT_CFG, loop)
    # activations of a single Linear are its inputs: amax exact on both sides
    assert torch.equal(m.input_quantizer.amax.cpu(), t["input_amax"])
    assert torch.equal(m.weight_quantizer.amax.cpu(), t["weight_amax"])
    out = m(t["test"].to(gpu)).detach().cpu()
    torch.testing.assert_close(out, t["out"], rtol=1e-5, atol=2e-5)  # fp32 GEMM order only


def _tiny_llama():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=32, max_position_embeddings=64)
    return LlamaForCausalLM(cfg).eval()


def test_c2_tiny_llama_fp8(gpu, monkeypatch):
    """Weight amax bit-exact vs the reference run; activation amax bit-exact vs torch's max|x| over
    the very tensors each quantizer collected on the GPU, and within rtol 1e-5 of the reference's
    (its CPU fp32 forward vs the GPU's GEMM / SDPA summation order)."""
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.calib.max import MaxCalibrator

    t = load_file(str(G / "llama_fp8.safetensors"))
    model = _tiny_llama()
    model.load_state_dict({k[3:]: v for k, v in t.items() if k.startswith("sd.")})
    model.to(gpu)
    ids = t["calib_ids"].to(gpu)

    def loop(mm):
        for b in ids:
            mm(b)

    seen = {}
    orig = MaxCalibrator.collect

    def spy(self, x):
        if self._axis is None and x.numel():
            a = x.detach().abs().amax().float()
            seen[id(self)] = torch.maximum(seen[id(self)], a) if id(self) in seen else a
        return orig(self, x)

    monkeypatch.setattr(MaxCalibrator, "collect", spy)
    mtq.quantize(model, mtq.FP8_DEFAULT_CFG, loop)
    monkeypatch.setattr(MaxCalibrator, "collect", orig)
    qs = {n: q for n, q in model.named_modules() if isinstance(q, mtq.TensorQuantizer) and q.amax is not None}
    got = {n: q.amax for n, q in qs.items()}
    want = {k[5:]: v for k, v in t.items() if k.startswith("amax.")}
    assert set(got) == set(want)
    self_checked = 0
    for n, v in want.items():
        if id(qs[n]._calibrator) in seen:
            assert torch.equal(got[n].float().reshape(()), seen[id(qs[n]._calibrator)].to(got[n].dtype).float()), n
            self_checked += 1
        if "weight_quantizer" in n:
            assert torch.equal(got[n].cpu(), v), n
        else:
            torch.testing.assert_close(got[n].cpu(), v, rtol=1e-5, atol=1e-6)
    assert self_checked >= len([n for n in want if "input_quantizer" in n])
    logits = model(t["test_ids"].to(gpu)).logits.detach().cpu()
    torch.testing.assert_close(logits, t["logits"], rtol=2e-3, atol=2e-3)


def test_c2_layerwise_matches_whole_model(gpu):
    """layerwise max calibration (qdq_from_prev False) reproduces the reference whole-model amax."""
    import modelopt_amd.torch.quantization as mtq

    t = load_file(str(G / "llama_fp8.safetensors"))
    model = _tiny_llama()
    model.load_state_dict({k[3:]: v for k, v in t.items() if k.startswith("sd.")})
    model.to(gpu)
    ids = t["calib_ids"].to(gpu)

    def loop(mm):
        for b in ids:
            mm(b)

    cfg = {**mtq.FP8_DEFAULT_CFG, "algorithm": {"method": "max", "layerwise": {"enable": True}}}
    mtq.quantize(model, cfg, loop)
    got = {n: q.amax for n, q in model.named_modules() if isinstance(q, mtq.TensorQuantizer) and q.amax is not None}
    want = {k[5:]: v for k, v in t.items() if k.startswith("amax.")}
    assert set(got) == set(want)
    for n, v in want.items():
        if "weight_quantizer" in n:
            assert torch.equal(got[n].cpu(), v), n
        else:
            torch.testing.assert_close(got[n].cpu(), v, rtol=1e-5, atol=1e-6)
    logits = model(t["test_ids"].to(gpu)).logits.detach().cpu()
    torch.testing.assert_close(logits, t["logits"], rtol=2e-3, atol=2e-3)


def _tiny_mixtral():
    from transformers import MixtralConfig, MixtralForCausalLM

    cfg = MixtralConfig(hidden_size=32, intermediate_size=48, num_hidden_layers=2, num_attention_heads=4,
                        num_key_value_heads=2, vocab_size=32, max_position_embeddings=64,
                        num_local_experts=4, num_experts_per_tok=2)
    return MixtralForCausalLM(cfg).eval()


def test_c5_tiny_mixtral_fp8_fused_experts(gpu):
    """C5 model class: transformers-5 fused experts through _QuantFusedExperts.  Per-expert weight
    amax bit-exact; activation amax / logits within the GEMM-order tolerance of test_c2."""
    import modelopt_amd.torch.quantization as mtq

    t = load_file(str(G / "mixtral_fp8.safetensors"))
    model = _tiny_mixtral()
    model.load_state_dict({k[3:]: v for k, v in t.items() if k.startswith("sd.")})
    model.to(gpu)
    ids = t["calib_ids"].to(gpu)

    def loop(mm):
        for b in ids:
            mm(b)

    mtq.quantize(model, mtq.FP8_DEFAULT_CFG, loop)
    got = {n: q.amax for n, q in model.named_modules() if isinstance(q, mtq.TensorQuantizer) and q.amax is not None}
    want = {k[5:]: v for k, v in t.items() if k.startswith("amax.")}
    assert set(got) == set(want)
    for n, v in want.items():
        if "weight_quantizer" in n:
            assert torch.equal(got[n].cpu(), v), n
        else:
            torch.testing.assert_close(got[n].cpu(), v, rtol=1e-5, atol=1e-6)
    logits = model(t["test_ids"].to(gpu)).logits.detach().cpu()
    torch.testing.assert_close(logits, t["logits"], rtol=2e-3, atol=2e-3)


class _SimpleMLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 16), nn.ReLU(), nn.Linear(16, 16))

    def forward(self, x):
        return self.net(x)


def test_c3_awq_lite(gpu):
    import modelopt_amd.torch.quantization as mtq

    t = load_file(str(G / "awq.safetensors"))
    meta = json.loads((G / "awq.json").read_text())
    model = _SimpleMLP()
    model.load_state_dict({k[3:]: v for k, v in t.items() if k.startswith("sd.")})
    model.to(gpu)
    data = [t[f"data{i}"].to(gpu) for i in range(4)]
    cfg = {
        "quant_cfg": [
            {"quantizer_name": "*", "enable": False},
            {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4, "block_sizes": {-1: 8, "type": "static"}}},
        ],
        "algorithm": {"method": "awq_lite", "alpha_step": 0.1, "debug": True},
    }

    def loop(mm):
        for d in data:
            mm(d)

    mtq.quantize(model, cfg, loop)
    for n, m in model.named_modules():
        if not hasattr(m, "awq_lite"):
            continue
        assert m.awq_lite.best_alpha == pytest.approx(meta[n]["best_alpha"]), n
        torch.testing.assert_close(m.awq_lite.best_scale.cpu(), t[f"best_scale.{n}"], rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(m.weight.detach().cpu(), t[f"weight.{n}"], rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(m.weight_quantizer.amax.cpu(), t[f"wamax.{n}"], rtol=1e-4, atol=1e-6)
    out = model(t["test"].to(gpu)).detach().cpu()
    torch.testing.assert_close(out, t["out"], rtol=1e-3, atol=1e-4)


def test_weight_collect_once_per_version(gpu):
    """A weight is reduced once per calibration even though forward_loop touches it every batch
    (the reference re-reduces it per batch); an in-place update makes it collect again."""
    from modelopt_amd.torch.quantization.calib import MaxCalibrator

    c = MaxCalibrator()
    w = nn.Parameter(torch.randn(64, 64, device=gpu))
    c.collect(w)
    a0 = c.compute_amax().clone()
    c.collect(w)  # same object, same version: skipped (same result either way)
    assert torch.equal(c.compute_amax(), a0)
    with torch.no_grad():
        w.mul_(2)
    c.collect(w)
    assert torch.equal(c.compute_amax(), a0 * 2)


@pytest.mark.parametrize("axis", [None, -1])
def test_shared_input_collect_matches_independent(gpu, axis):
    """Calibrators that collect the very same tensor (q/k/v_proj input quantizers) share one
    reduction from the second batch on; every running max must equal an unshared collect,
    including when the shared tensor is modified in place between siblings (NaN included)."""
    from modelopt_amd.torch.quantization.calib import MaxCalibrator
    from oracle import ref_ops as R

    cs = [MaxCalibrator(axis=axis) for _ in range(3)]
    lone = MaxCalibrator(axis=axis)
    g = torch.Generator().manual_seed(7)
    seen = [[] for _ in range(3)]
    for step in range(5):
        x = (torch.randn(64, 256, generator=g) * (step + 1)).to(torch.bfloat16).to(gpu)
        for i, c in enumerate(cs):
            if step == 3 and i == 2:
                x.mul_(3)  # in place between siblings: the third must reduce it again
            if step == 4 and i == 1:
                x[5, 7] = float("nan")
            c.collect(x)
            seen[i].append(x.clone().cpu())
        lone.collect(torch.randn(64, 256, device=gpu).to(torch.bfloat16))  # interleaved other tensor
    assert cs[0]._share  # the first calibrator became the producer
    raxis = None if axis is None else [0]
    for i, c in enumerate(cs):
        want = torch.stack([R.reduce_amax(t, axis=raxis).float().reshape(-1) for t in seen[i]]).amax(0)
        got = c._acc.cpu()
        assert torch.equal(torch.isnan(got), torch.isnan(want)), i
        ok = ~torch.isnan(want)
        assert torch.equal(got[ok], want[ok]), i
