"""End-to-end parity at production dispatch sizes.

``mtq.quantize`` on the GPU against the reference run on the CPU (``tests/golden/prod.*``,
``tests/golden/make_golden.py gen_prod``) for models whose linears have Llama-3-8B's shapes, so the
kernels the bench and C2 / C3 run are the ones compared end to end:

* a 2-layer Llama (hidden 4096, intermediate 14336, 32 / 8 heads, bf16) under FP8_DEFAULT_CFG
  (per-tensor amax: ``amax_persist``), INT8_DEFAULT_CFG (per-channel weights: ``amax_rows_u``,
  ``ew_rowwave``) and INT4_AWQ_CFG (awq_lite, block 128: the fused ``awq_search_w4`` search on
  k/v/q/o/gate/up, the batched library path on down, ``ew_group_sk`` for the promoted static-block
  weights);
* a Mixtral layer at hidden 1024 with 8 experts (the fused-experts plugin) under FP8_DEFAULT_CFG.

The weights are regenerated from the seed (``tests/golden/prod_models.py``) and checked against the
reference run's sha256 fingerprint first.  Criteria:
* weight amax: bit-exact (they depend on the weights alone);
* activation amax: bit-exact against torch's max|x| over the very tensors each quantizer collected
  on the GPU; against the reference within 2 bf16 ulps -- the reference computes them from its CPU
  bf16 forward, this build from the GPU's (hipBLASLt GEMM, SDPA, RMSNorm reductions in another
  order), and the layer-1 MLP activations measured 1-2 ulps apart -- with the bit-equal count
  reported;
* AWQ: the same best alpha on all but at most 2 of the 14 linears; act_scale rtol 2e-2 (the means
  follow the reference CPU run's summation order, r06, but over activations that differ as
  above), best scales rtol 2e-2 where the alpha agrees and bit-exact where the act_scale is too; the static-block weight amax bit-equal count is reported (a 1-ulp act_scale
  difference changes the scale and so the block amax);
* logits: against a noise floor measured in the test -- the same GPU forward with the reference
  run's amax loaded into the quantizers.  The remaining distance is the GPU-vs-CPU bf16 forward
  amplified by FP8 rounding flips (r05a: cosine 0.9979 for llama_fp8); this build's own amax may
  cost at most twice that distance (a 1-ulp amax difference moves an FP8 scale).
The launches per kernel family (``_ext.dispatch_counts``, the library's dispatch registry) are
asserted, so the test fails if the production shapes stop reaching those kernels.
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

G = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(G))
from prod_models import PROD_CASES, fingerprint, prod_inputs, prod_model, sha  # noqa: E402

# kernel families each case must reach (modelopt_amd._ext.dispatch_counts, mtq_dispatch_counts)
EXPECTED_KERNELS = {
    "llama_fp8": ["amax_persist", "ew_vec"],
    "llama_int8": ["amax_persist", "amax_rows_u", "ew_rowwave"],
    "llama_int4_awq": ["awq_search_w4", "awq_prescale", "awq_mse_multi", "block_quant_dyn", "ew_group_sk"],
    "mixtral_fp8": ["amax_persist", "ew_vec"],
}


@pytest.fixture(scope="module")
def golden():
    from safetensors.torch import load_file

    return load_file(str(G / "prod.safetensors")), json.loads((G / "prod.json").read_text())


def _run(name, gpu, monkeypatch):
    import copy

    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd import _ext
    from modelopt_amd.torch.quantization.calib.max import MaxCalibrator

    kind, seed, cfg_name, algo = PROD_CASES[name]
    model = prod_model(kind, seed)
    fp = fingerprint(model)
    model = model.to(gpu)
    ids, test = prod_inputs(seed)
    cfg = copy.deepcopy(getattr(mtq, cfg_name))
    if algo is not None:
        cfg["algorithm"] = algo

    # every per-tensor max collect's own input, reduced by torch on the GPU: the product's amax
    # must equal it bit for bit (the kernel dispatch at these shapes, independent of the
    # CPU-vs-GPU forward differences the reference comparison sees)
    seen: dict[int, torch.Tensor] = {}
    orig_collect = MaxCalibrator.collect

    def spy(self, x):
        if self._axis is None and x.numel() and not x.is_meta:
            a = x.detach().abs().amax().float()
            seen[id(self)] = torch.maximum(seen[id(self)], a) if id(self) in seen else a
        return orig_collect(self, x)

    monkeypatch.setattr(MaxCalibrator, "collect", spy)

    def loop(mm):
        for b in ids:
            mm(b.to(gpu))

    before = _ext.dispatch_counts()
    with torch.no_grad():
        mtq.quantize(model, cfg, loop)
        logits = model(test.to(gpu)).logits.float().cpu()
    torch.cuda.synchronize()
    after = _ext.dispatch_counts()
    monkeypatch.setattr(MaxCalibrator, "collect", orig_collect)
    launched = {k: after[k] - before[k] for k in after if after[k] > before[k]}
    return model, fp, logits, launched, seen, test


def _ulps(got: torch.Tensor, want: torch.Tensor) -> torch.Tensor:
    """|got - want| in bf16 ulps of want (8 significand bits: ulp = 2^(e - 7))."""
    g, w = got.float(), want.float()
    e = torch.floor(torch.log2(w.abs().clamp_min(1e-30)))
    return (g - w).abs() / torch.exp2(e - 7)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", list(PROD_CASES))
def test_prod_e2e(gpu, golden, name, monkeypatch):
    import modelopt_amd.torch.quantization as mtq

    t, meta = golden
    m = meta[name]
    model, fp, logits, launched, seen, test = _run(name, gpu, monkeypatch)
    assert fp == m["fingerprint"], "regenerated weights differ from the reference run's"
    print(f"{name}: library launches {launched}")
    missing = [k for k in EXPECTED_KERNELS[name] if not launched.get(k)]
    assert not missing, f"expected kernel families not dispatched: {missing}"

    quantizers = {n: q for n, q in model.named_modules()
                  if isinstance(q, mtq.TensorQuantizer) and q.is_enabled and q.amax is not None}
    want_names = {k[len(name) + 6:] for k in t if k.startswith(f"{name}.amax.")} | set(m["amax_sha"])
    assert set(quantizers) == want_names
    awq = m["awq"]
    exact_act = n_act = exact_awq = self_checked = 0
    worst = 0.0
    for n, q in quantizers.items():
        a = q.amax.detach().cpu()
        cal = q._calibrator
        if id(cal) in seen:  # the product's amax vs torch on the very tensors it collected
            assert torch.equal(a.reshape(()).float(), seen[id(cal)].cpu().to(a.dtype).float()), n
            self_checked += 1
        lin = n.rsplit(".", 1)[0]
        if lin in awq:  # AWQ static-block weight amax: depends on the searched scale
            ref_sha = m["amax_sha"][n][0] if n in m["amax_sha"] else sha(t[f"{name}.amax.{n}"])
            exact_awq += int(sha(a) == ref_sha)
            continue
        w = t[f"{name}.amax.{n}"]
        assert a.shape == w.shape and a.dtype == w.dtype, n
        if n.endswith("weight_quantizer"):
            assert torch.equal(a, w), f"{n}: weight amax not bit-exact"
        else:
            u = float(_ulps(a, w).max())
            worst = max(worst, u)
            assert u <= 2, f"{n}: activation amax {u} bf16 ulps from the reference: {a.flatten()[:4]} vs {w.flatten()[:4]}"
            exact_act += int(torch.equal(a, w))
            n_act += 1
    assert self_checked >= n_act, (self_checked, n_act)
    print(f"{name}: {self_checked} per-tensor amax bit-equal to torch on the collected tensors; "
          f"activation amax vs reference bit-equal {exact_act}/{n_act}, worst {worst:.0f} ulp")

    if awq:
        same = act_equal = 0
        for lin, info in awq.items():
            h = model.get_submodule(lin).awq_lite
            ra, rb = t[f"{name}.act_scale.{lin}"], t[f"{name}.best_scale.{lin}"]
            torch.testing.assert_close(h.act_scale.cpu(), ra, rtol=2e-2, atol=1e-6)
            same += int(h.best_alpha == info["best_alpha"])
            if h.best_alpha == info["best_alpha"]:
                if torch.equal(h.act_scale.cpu().view(torch.int32), ra.view(torch.int32)):
                    # same statistics in, same scale out: the table follows the reference CPU run's
                    # operations (csrc/mtq_awq_scale.hip) -- bit-exact
                    act_equal += 1
                    assert torch.equal(h.best_scale.cpu().view(torch.int32), rb.view(torch.int32)), lin
                torch.testing.assert_close(h.best_scale.cpu(), rb, rtol=2e-2, atol=0)
        print(f"{name}: best alpha equal on {same}/{len(awq)} linears; act_scale bit-equal (so best_scale "
              f"asserted bit-exact) on {act_equal}; static-block amax bit-equal on {exact_awq}/{len(awq)}")
        assert same >= len(awq) - 2, f"best alpha differs on {len(awq) - same} of {len(awq)} linears"

    ref = t[f"{name}.logits"]

    def dist(lg):
        err = (lg - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
        cos = torch.nn.functional.cosine_similarity(lg.flatten(), ref.flatten(), dim=0).item()
        return err, cos

    # noise floor: the same GPU forward with the reference run's own amax loaded into every
    # quantizer it holds one for -- what remains is the GPU-vs-CPU bf16 forward (GEMM / SDPA /
    # RMSNorm order), amplified by FP8 rounding flips, not this build's calibration
    saved = {}
    for n, q in quantizers.items():
        key = f"{name}.amax.{n}"
        if key in t:
            saved[n] = q.amax.detach().clone()
            q.amax = t[key].to(q.amax.device)
    with torch.no_grad():
        floor_logits = model(test.to(gpu)).logits.float().cpu()
    for n, a in saved.items():
        quantizers[n].amax = a
    err, cos = dist(logits)
    ferr, fcos = dist(floor_logits)
    print(f"{name}: logits max rel err {err:.3e}, cosine {cos:.6f}; with the reference amax loaded "
          f"({len(saved)} quantizers): {ferr:.3e}, {fcos:.6f}")
    assert fcos > 0.99 and ferr < 0.2, "GPU forward with the reference's amax far from the reference logits"
    # this build's amax cost at most twice the forward's own distance (plus a small absolute slack)
    assert 1 - cos <= 2 * (1 - fcos) + 5e-4, (cos, fcos)
    assert err <= 2 * ferr + 0.02, (err, ferr)
