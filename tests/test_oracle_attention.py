"""The attention oracle (oracle/attention_ref.py) vs the reference's own Triton flash attention
with softmax-P qdq (tests/golden/attention.*, tests/golden/make_golden_attention.py).  CPU only.

Tolerance: the golden is the interpreter's fp32 numpy arithmetic (matmul summation order);
the oracle sums P . V in float64 then rounds, so an output element can land one output-dtype
ulp away.  Measured: >= 99.97 % of the elements bit-identical in every case, 5 of 9 cases
entirely, the largest difference one ulp (4.9e-4 at |o| ~ 2 in bf16).  The test asserts
>= 99.9 % identical and every difference within 2 ulp of the output dtype."""

import json
from pathlib import Path

import pytest
import torch
from safetensors.torch import load_file

from oracle import attention_ref as A

G = Path(__file__).resolve().parent / "golden"
META = json.loads((G / "attention.json").read_text())


@pytest.fixture(scope="module")
def gold():
    return load_file(str(G / "attention.safetensors"))


def run_oracle(gold, name):
    mt = META[name]
    b, lq, lk = mt["batch"], mt["lens_q"], mt["lens_k"]
    sq, sk = max(lq), max(lk)
    kw = dict(b_start_loc=torch.arange(b) * sq, b_seq_len=torch.tensor(lq), is_causal=mt["causal"],
              softmax_scale=mt["d"] ** -0.5)
    kw.update(b_start_loc_k=torch.arange(b) * sk, b_seq_len_k=torch.tensor(lk))
    if mt["p_qdq"]:
        kw["p_qdq"] = mt["p_qdq"]
        if mt["amax"] is not None:
            kw["p_qdq_amax"] = mt["amax"]
    return A.attention_fwd(gold[f"{name}.q"], gold[f"{name}.k"], gold[f"{name}.v"], **kw)


@pytest.mark.parametrize("name", sorted(META))
def test_oracle_matches_reference_attention(gold, name):
    o = run_oracle(gold, name)
    want = gold[f"{name}.o"]
    assert o.dtype == want.dtype
    err = (o.float() - want.float()).abs()
    ulp = torch.finfo(want.dtype).eps * torch.maximum(want.float().abs(), torch.tensor(2.0 ** -6))
    assert bool((err <= 2 * ulp).all()), float((err / ulp).max())
    assert float((err == 0).float().mean()) >= 0.999


def test_p_qdq_changes_the_result(gold):
    """The P quantisation is not a no-op: FP8 / NVFP4 differ from the unquantised attention."""
    name = "bf16_d64_fp8"
    plain = dict(META[name], p_qdq=None)
    META["_plain"] = plain
    try:
        for k in ("q", "k", "v"):
            gold[f"_plain.{k}"] = gold[f"{name}.{k}"]
        o0 = run_oracle(gold, "_plain")
    finally:
        del META["_plain"]
    assert (o0.float() - gold[f"{name}.o"].float()).abs().max() > 1e-2
