"""Histogram calibrator host logic against the reference run (no GPU): the MSE / percentile /
entropy amax computed from the reference's own collected histograms (``tests/golden/calib_ref.*``,
``make_golden.py gen_calib_ref``) must equal the amax the reference computed from them, including
the MSE sweep's ``fake_tensor_quant(centers, amax, num_bits, unsigned)`` call as it binds
(calib/histogram.py:305-312 -> tensor_quant.py:350-394, 607-645) and the (4, 3) TypeError."""

import json
from pathlib import Path

import pytest
import torch
from safetensors.torch import load_file

G = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def ref():
    return load_file(str(G / "calib_ref.safetensors")), json.loads((G / "calib_ref.json").read_text())


def test_amax_methods_from_reference_histograms(ref):
    from modelopt_amd.torch.quantization.calib import histogram as H

    t, meta = ref
    for c in meta["cases"]:
        hist = t[f"hist_{c['key']}"].int().numpy()
        edges = t[f"edges_{c['key']}"].numpy()
        assert float(H._compute_amax_mse(hist, edges, 8, False)) == c["mse"], c["key"]
        assert float(H._compute_amax_percentile(hist, edges, 99.99)) == c["percentile_9999"], c["key"]
        if "entropy" in c:
            assert float(H._compute_amax_entropy(hist.copy(), edges, 8, False)) == c["entropy"], c["key"]


def test_mse_reference_call_semantics():
    """num_bits lands in ``bias`` and ``unsigned`` in ``num_bits``: 0 bits -> every centre maps to
    amax + 8 (clamp with min 0.5 > max -0.5), 1 bit -> 0 / 0 = NaN; a tiny amax -> bias - 0.5."""
    from modelopt_amd.torch.quantization.calib import histogram as H

    c = torch.linspace(0, 4, 9)
    q0 = H._reference_call_qdq(c, torch.tensor(2.0), 8, 0)
    assert torch.equal(q0, torch.full_like(c, 10.0))
    q1 = H._reference_call_qdq(c, torch.tensor(2.0), 8, 1)
    assert torch.isnan(q1).all()
    qt = H._reference_call_qdq(c, torch.tensor(1e-9), 8, 0)
    assert torch.equal(qt, torch.full_like(c, 7.5))


def test_mse_fp8_raises_like_reference(ref, monkeypatch):
    from modelopt_amd.torch.quantization.calib import histogram as H

    _, meta = ref
    hist = torch.arange(256).int().numpy()
    edges = torch.linspace(0, 1, 257).numpy()
    with pytest.raises(TypeError) as e:
        H._compute_amax_mse(hist, edges, (4, 3), False, start_bin=16)
    assert "TypeError: " + str(e.value) == meta["fp8_mse_error"]
    monkeypatch.setenv("MTQ_AMD_HIST_MSE", "intent")  # the documented-intent opt-in quantises FP8
    assert H._compute_amax_mse(hist, edges, (4, 3), False, start_bin=16) is not None


def test_oracle_mse_matches_reference_run(ref):
    from oracle import ref_ops as R

    t, meta = ref
    for c in meta["cases"]:
        hist = t[f"hist_{c['key']}"].int().numpy()
        edges = t[f"edges_{c['key']}"].numpy()
        assert float(R.compute_amax_mse(hist, edges, 8, False)) == c["mse"], c["key"]


def test_histc_thread_count_in_quantizer_state():
    """The histogram calibrator's recorded chunk count travels with the quantizer state (the GPU
    test test_gpu_hist_ref.py::test_histc_thread_count_is_recorded_and_restored checks the counts)."""
    from modelopt_amd.torch.quantization import TensorQuantizer
    from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig

    q = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, calibrator="histogram"))
    assert q._calibrator._histc_threads is None
    assert "_histc_threads" not in q.get_modelopt_state()
    q._calibrator._histc_threads = 5
    state = q.get_modelopt_state()
    assert state["_histc_threads"] == 5
    r = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, calibrator="histogram"))
    r.set_from_modelopt_state(state)
    assert r._calibrator._histc_threads == 5
    assert "_histc_threads" not in r.__dict__
    m = TensorQuantizer(QuantizerAttributeConfig(num_bits=8))  # max calibrator: the key is ignored
    m.set_from_modelopt_state(state)
    assert not hasattr(m._calibrator, "_histc_threads")


def test_hist_threads_env_override(monkeypatch):
    """MTQ_AMD_HIST_THREADS fixes the chunk count a new histogram calibrator records."""
    from modelopt_amd.torch.quantization.calib import histogram

    monkeypatch.setenv("MTQ_AMD_HIST_THREADS", "5")
    assert histogram._histc_threads() == 5
    monkeypatch.delenv("MTQ_AMD_HIST_THREADS")
    assert histogram._histc_threads() == max(1, torch.get_num_threads())
