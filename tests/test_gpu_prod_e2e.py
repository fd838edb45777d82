"""End-to-end parity at production dispatch sizes.

``mtq.quantize`` on the GPU against the reference run on the CPU (``tests/golden/prod.*``,
``tests/golden/make_golden.py gen_prod``) for models whose linears have Llama-3-8B's shapes, so the
kernels the bench and C2 / C3 run are the ones compared end to end:

* a 2-layer Llama (hidden 4096, intermediate 14336, 32 / 8 heads, bf16) under FP8_DEFAULT_CFG
  (per-tensor amax: ``amax_persist``), INT8_DEFAULT_CFG (per-channel weights: ``amax_rows_u``,
  ``ew_rowwave``) and INT4_AWQ_CFG (awq_lite, block 128: the fused ``awq_search_pp`` search on
  k/v (N = 1024), the batched library path on q/o/gate/up/down, ``ew_group_sk`` for the promoted
  static-block weights);
* a Mixtral layer at hidden 1024 with 8 experts (the fused-experts plugin) under FP8_DEFAULT_CFG.

The weights are regenerated from the seed (``tests/golden/prod_models.py``) and checked against the
reference run's sha256 fingerprint first.  Criteria:
* weight amax: bit-exact (they depend on the weights alone);
* activation amax: the reference computes them from its CPU bf16 forward, this build from the GPU's
  (hipBLASLt GEMM, SDPA, RMSNorm reductions in another order), so a bf16 activation may round the
  other way: each amax within 1 bf16 ulp (rel 2^-8), and the test reports how many are bit-equal;
* AWQ: the same best alpha per linear where the reference's loss margin to the runner-up is not a
  near-tie; act_scale rtol 2e-2 (means of |x| over the same bf16-rounded activations); for the
  linears whose alpha and act_scale inputs agree exactly (the first layer reads the embedding
  through RMSNorm), the static-block weight amax bit-exact by sha256;
* logits: close at a bf16-GEMM tolerance (2-layer stack).
The kernel names of each case are collected with the torch profiler and the expected dispatch is
asserted, so the test fails if the production-size shapes stop reaching those kernels.
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

EXPECTED_KERNELS = {
    "llama_fp8": ["amax_persist_kernel"],
    "llama_int8": ["amax_rows_u_kernel", "ew_rowwave_kernel"],
    "llama_int4_awq": ["awq_search_pp_kernel", "ew_group_sk_kernel", "block_quant_dyn_kernel"],
    "mixtral_fp8": ["amax_persist_kernel", "mask_rows_kernel"],
}


@pytest.fixture(scope="module")
def golden():
    from safetensors.torch import load_file

    return load_file(str(G / "prod.safetensors")), json.loads((G / "prod.json").read_text())


def _run(name, gpu):
    import copy

    import modelopt_amd.torch.quantization as mtq

    kind, seed, cfg_name, algo = PROD_CASES[name]
    model = prod_model(kind, seed)
    fp = fingerprint(model)
    model = model.to(gpu)
    ids, test = prod_inputs(seed)
    cfg = copy.deepcopy(getattr(mtq, cfg_name))
    if algo is not None:
        cfg["algorithm"] = algo

    def loop(mm):
        for b in ids:
            mm(b.to(gpu))

    from torch.profiler import ProfilerActivity, profile

    with torch.no_grad(), profile(activities=[ProfilerActivity.CUDA]) as prof:
        mtq.quantize(model, cfg, loop)
        logits = model(test.to(gpu)).logits.float().cpu()
        torch.cuda.synchronize()
    kernels = {e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA}
    return model, fp, logits, kernels


def _ulp_ok(got: torch.Tensor, want: torch.Tensor) -> torch.Tensor:
    g, w = got.float(), want.float()
    return (g - w).abs() <= w.abs() * 2.0**-8 + 1e-30


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", list(PROD_CASES))
def test_prod_e2e(gpu, golden, name):
    import modelopt_amd.torch.quantization as mtq

    t, meta = golden
    m = meta[name]
    model, fp, logits, kernels = _run(name, gpu)
    assert fp == m["fingerprint"], "regenerated weights differ from the reference run's"
    missing = [k for k in EXPECTED_KERNELS[name] if not any(k in n for n in kernels)]
    print(f"{name}: {len(kernels)} distinct kernels; library kernels:",
          sorted({n.split('<')[0].split('(')[0].replace('void ', '') for n in kernels
                  if any(s in n for s in ('amax_', 'ew_', 'awq_', 'mask_rows', 'block_quant'))}))
    assert not missing, f"expected kernels not dispatched: {missing}"

    quantizers = {n: q for n, q in model.named_modules()
                  if isinstance(q, mtq.TensorQuantizer) and q.is_enabled and q.amax is not None}
    want_names = {k[len(name) + 6:] for k in t if k.startswith(f"{name}.amax.")} | set(m["amax_sha"])
    assert set(quantizers) == want_names
    awq = m["awq"]
    exact_act = near_act = 0
    exact_awq = 0
    for n, q in quantizers.items():
        a = q.amax.detach().cpu()
        lin = n.rsplit(".", 1)[0]
        if lin in awq:  # AWQ static-block weight amax: depends on the chosen scale
            same_alpha = model.get_submodule(lin).awq_lite.best_alpha == awq[lin]["best_alpha"]
            ref_sha = m["amax_sha"][n][0] if n in m["amax_sha"] else sha(t[f"{name}.amax.{n}"])
            if same_alpha and lin.startswith("model.layers.0.self_attn"):
                assert sha(a) == ref_sha, f"{n}: static block amax differs"
            exact_awq += int(sha(a) == ref_sha)
            continue
        w = t[f"{name}.amax.{n}"]
        assert a.shape == w.shape and a.dtype == w.dtype, n
        if n.endswith("weight_quantizer"):
            assert torch.equal(a, w), f"{n}: weight amax not bit-exact"
        else:
            ok = _ulp_ok(a, w)
            assert bool(ok.all()), f"{n}: activation amax beyond 1 bf16 ulp: {a.flatten()[:4]} vs {w.flatten()[:4]}"
            exact_act += int(torch.equal(a, w))
            near_act += 1
    if awq:
        print(f"{name}: AWQ block amax bit-equal on {exact_awq}/{len(awq)} linears")
    print(f"{name}: activation amax bit-equal {exact_act}/{near_act}")

    if awq:
        same = 0
        for lin, info in awq.items():
            h = model.get_submodule(lin).awq_lite
            torch.testing.assert_close(h.act_scale.cpu(), t[f"{name}.act_scale.{lin}"], rtol=2e-2, atol=1e-6)
            same += int(h.best_alpha == info["best_alpha"])
            if h.best_alpha == info["best_alpha"]:
                torch.testing.assert_close(h.best_scale.cpu(), t[f"{name}.best_scale.{lin}"], rtol=2e-2, atol=0)
        print(f"{name}: best alpha equal on {same}/{len(awq)} linears")
        assert same >= len(awq) - 2, f"best alpha differs on {len(awq) - same} of {len(awq)} linears"

    ref = t[f"{name}.logits"]
    err = (logits - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
    print(f"{name}: logits max rel err {err:.3e}")
    assert err < 5e-2
