"""HistogramCalibrator on the GPU against the reference run at > 2^24 counts per call.

Golden ``tests/golden/calib_ref.*`` (``make_golden.py gen_calib_ref``): the reference's
``HistogramCalibrator.collect`` (calib/histogram.py:77-130, torch.histc's fp32 counts) on two
40 M-element peaked bf16 tensors (``hist_inputs.peaked``: one bin past 2^24 in each call) with 1
and 3 intra-op threads and with skip_zeros, then ``compute_amax`` (entropy / percentile / MSE).
The product sets the same thread count (``torch.set_num_threads``), counts each thread's chunk
exactly on the GPU and folds them as histc does: histograms and amax must be bit-equal.  The
small-batch MSE cases pin the MSE sweep's actual call (``bias = num_bits``).
"""

import json
import sys
from pathlib import Path

import pytest
import torch
from safetensors.torch import load_file

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(G))


def test_histogram_calibrator_matches_reference_above_2p24(gpu):
    from hist_inputs import peaked
    from modelopt_amd.torch.quantization.calib import HistogramCalibrator

    t = load_file(str(G / "calib_ref.safetensors"))
    meta = json.loads((G / "calib_ref.json").read_text())
    saved = torch.get_num_threads()
    try:
        for c in meta["cases"]:
            torch.set_num_threads(c["threads"])
            h = HistogramCalibrator(8, None, False, num_bins=2048, skip_zeros=c["skip_zeros"])
            for scale in (1.0, 1.5):
                h.collect(peaked(scale=scale, zeros_every=4 if c["skip_zeros"] else 0).to(gpu))
            assert h._num_bins == c["num_bins"], c["key"]
            got = h._calib_hist.cpu()
            want = t[f"hist_{c['key']}"]
            assert torch.equal(h._calib_bin_edges.cpu(), t[f"edges_{c['key']}"]), c["key"]
            assert torch.equal(got, want), (c["key"], (got - want).abs().max().item())
            assert float(got.max()) == c["max_count"]
            assert float(h.compute_amax("percentile", percentile=99.99)) == c["percentile_9999"], c["key"]
            assert float(h.compute_amax("mse")) == c["mse"], c["key"]
            if "entropy" in c:
                assert float(h.compute_amax("entropy")) == c["entropy"], c["key"]
    finally:
        torch.set_num_threads(saved)


def test_histogram_mse_small_batches_match_reference(gpu):
    from modelopt_amd.torch.quantization.calib import HistogramCalibrator

    meta = json.loads((G / "calib_ref.json").read_text())
    g = torch.Generator().manual_seed(20)
    xs = [torch.randn(32, 64, generator=g) * s for s in (1.0, 2.5, 0.7)]
    for nb, u in [(8, False), (8, True), (4, False)]:
        h = HistogramCalibrator(nb, None, u, num_bins=256)
        for x in xs:
            h.collect((x.abs() if u else x).to(gpu))
        assert float(h.compute_amax("mse", start_bin=16)) == meta[f"small_mse_b{nb}_u{int(u)}"], (nb, u)
    h = HistogramCalibrator((4, 3), None, False, num_bins=256)
    h.collect(xs[0].to(gpu))
    with pytest.raises(TypeError):
        h.compute_amax("mse", start_bin=16)


def test_histc_thread_count_is_recorded_and_restored(gpu):
    """the >2^24 emulation's chunk count is fixed at the first collect and
    saved with the quantizer state; a quantizer restored from that state in a process with a
    different intra-op thread count counts exactly as the recording one (the reference run with 3
    threads, golden case t3_skip0)."""
    from hist_inputs import peaked
    from modelopt_amd.torch.quantization import TensorQuantizer
    from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig

    t = load_file(str(G / "calib_ref.safetensors"))
    xs = [peaked(scale=s).to(gpu) for s in (1.0, 1.5)]
    saved = torch.get_num_threads()
    try:
        torch.set_num_threads(3)
        q = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, calibrator="histogram"))
        q.disable_quant()
        q.enable_calib()
        q(xs[0])
        state = q.get_modelopt_state()
        assert state["_histc_threads"] == 3
        torch.set_num_threads(1)
        r = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, calibrator="histogram"))
        r.set_from_modelopt_state(state)
        r.disable_quant()
        r.enable_calib()
        assert r._calibrator._histc_threads == 3
        for x in xs:
            r(x)
        assert torch.equal(r._calibrator._calib_hist.cpu(), t["hist_t3_skip0"])
        # a fresh calibrator in this process records its own count (1) and matches the 1-thread run
        f = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, calibrator="histogram"))
        f.disable_quant()
        f.enable_calib()
        for x in xs:
            f(x)
        assert f._calibrator._histc_threads == 1
        assert torch.equal(f._calibrator._calib_hist.cpu(), t["hist_t1_skip0"])
    finally:
        torch.set_num_threads(saved)


def test_histc_exact_counts_mode(gpu, monkeypatch):
    """MTQ_AMD_HIST_COUNTS=exact: one launch with exact integer counts even when a bin passes 2^24
    in one call (torch.histc's fp32 counts stop at 2^24 there)."""
    from hist_inputs import peaked
    from modelopt_amd.torch.quantization.calib import HistogramCalibrator

    x = peaked(scale=1.0).to(gpu)
    monkeypatch.setenv("MTQ_AMD_HIST_COUNTS", "exact")
    h = HistogramCalibrator(8, None, False, num_bins=2048)
    h.collect(x)
    got = h._calib_hist.cpu()
    assert float(got.sum()) == float(x.numel())  # every element counted, no 2^24 saturation
    assert float(got.max()) > 2**24
    a = x.float().abs().flatten()
    want = torch.histc(a.cpu().double(), bins=2048, min=0, max=float(a.max()))
    assert torch.equal(got.double(), want)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_histc_chunked_single_launch_matches_per_chunk_counts(gpu, dtype):
    """histogram_abs_chunked (every chunk in one launch, rows summed in chunk order) against the
    per-chunk launches over slices: chunk edges off the 8-element vectors, uniform and explicit
    (skip_zeros-style) bounds, 1..300 chunks (more than 16: the fold adds its chunk groups in
    order; more than the CUs: one workgroup per chunk), a bin past 2^24 in the sum."""
    from modelopt_amd import _ext

    ops = _ext.ops()
    g = torch.Generator(device=gpu).manual_seed(3)
    n = 8 * 2_100_003
    x = (torch.randn(n, device=gpu, generator=g) * 2).to(dtype)
    x[::5] = 0
    x[7::11] = 0.25  # one heavy bin
    hmax = torch.tensor([6.0], device=gpu)
    F32 = 2**24

    def per_chunk(bounds, skip):
        h = torch.zeros(2048, device=gpu)
        for b, e in zip(bounds[:-1], bounds[1:]):
            c = torch.zeros(2048, dtype=torch.int32, device=gpu)
            if e > b:
                ops.histogram_abs_accumulate(x[b:e], hmax, c, 2048, skip)
            h += c.float().clamp_(max=F32)
        return h

    for chunks in (1, 3, 16, 17, 40, 300):
        chunk = -(-n // chunks)
        bounds = [min(t * chunk, n) for t in range(chunks)] + [n]
        for skip in (False, True):
            got = ops.histogram_abs_chunked(x, hmax, 2048, skip, None, chunk, chunks)
            assert torch.equal(got, per_chunk(bounds, skip)), (chunks, skip)
    # explicit device bounds, ragged (including an empty chunk)
    bounds = [0, 13, 13, 1_000_001, 9_999_999, n - 3, n]
    dev_b = torch.tensor(bounds, dtype=torch.int64, device=gpu)
    got = ops.histogram_abs_chunked(x, hmax, 2048, True, dev_b, 0, len(bounds) - 1)
    assert torch.equal(got, per_chunk(bounds, True))
    # 2^24 clamp: a single chunk holding > 2^24 elements of the heavy bin
    y = torch.full((F32 + 64,), 0.25, dtype=dtype, device=gpu)
    got = ops.histogram_abs_chunked(y, hmax, 2048, False, None, F32 + 64, 1)
    assert float(got.max()) == float(F32) and float(got.sum()) == float(F32)


def test_histc_chunked_scratch_any_contents_and_reusable(gpu):
    """The chunked histogram overwrites every per-workgroup row of its scratch, so a caller's
    buffer holding garbage, reused across calls with varying chunk counts / bins, gives the
    results of fresh-scratch calls; a buffer below mtq_histogram_chunked_scratch_words is
    replaced by a fresh one, not overrun."""
    from modelopt_amd import _ext

    ops = _ext.ops()
    g = torch.Generator(device=gpu).manual_seed(5)
    n = 8 * 1_500_001
    x = (torch.randn(n, device=gpu, generator=g) * 3).to(torch.bfloat16)
    hmax = torch.tensor([8.0], device=gpu)
    scratch = torch.randint(-2**31, 2**31 - 1, (1 << 22,), dtype=torch.int32, device=gpu, generator=g)
    small = torch.full((64,), 7, dtype=torch.int32, device=gpu)
    for chunks, bins in ((16, 2048), (3, 4096), (7, 1000), (16, 2048)):
        chunk = -(-n // chunks)
        fresh = ops.histogram_abs_chunked(x, hmax, bins, False, None, chunk, chunks)
        for _ in range(2):
            got = ops.histogram_abs_chunked(x, hmax, bins, False, None, chunk, chunks, scratch)
            assert torch.equal(got, fresh), (chunks, bins)
        assert torch.equal(ops.histogram_abs_chunked(x, hmax, bins, False, None, chunk, chunks, small), fresh)
        assert int((small != 7).sum()) == 0, "a too-small scratch was written"


def _host_nonzero_bounds(x, threads, grain=32768):
    """torch.histc's skip_zeros chunking restated on the host: T' = min(T, ceil(N / grain)),
    chunk = ceil(N / T'), chunk t starts at the input index of the (t * chunk)-th non-zero."""
    nz = torch.nonzero(x.view(-1).float() != 0).view(-1).cpu()
    kept, n = nz.numel(), x.numel()
    teff = min(threads, -(-kept // grain))
    chunk = -(-kept // teff) if teff else 1
    return [0] + [int(nz[t * chunk]) if t * chunk < kept else n for t in range(1, threads)] + [n]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_histc_nonzero_bounds_on_device(gpu, dtype):
    """skip_zeros chunking found on the device (histogram_abs_chunked_nonzero: per-tile non-zero
    counts, one block per boundary) against host-computed bounds fed to histogram_abs_chunked:
    scattered and clustered zeros, a zero-free and an all-zero input, -0, NaN (kept, as x != 0
    keeps it), T = 1, T past ceil(N / grain), a chunk boundary inside a vector."""
    from modelopt_amd import _ext

    ops = _ext.ops()
    g = torch.Generator(device=gpu).manual_seed(9)
    hmax = torch.tensor([6.0], device=gpu)
    n = 8 * 1_300_007
    base = (torch.randn(n, device=gpu, generator=g) * 2).to(dtype)
    cases = {}
    x = base.clone()
    x[::3] = 0
    x[5::7] = -0.0
    cases["scattered"] = x
    x = base.clone()
    x[: n // 3] = 0  # the first chunks' boundaries all fall in one zero run
    x[n // 2: n // 2 + 70_001] = 0
    x[123] = float("nan")
    cases["clustered"] = x
    cases["no_zeros"] = base.abs() + 0.01
    cases["all_zero"] = torch.zeros(n, dtype=dtype, device=gpu)
    x = torch.zeros(n, dtype=dtype, device=gpu)
    x[1000:1000 + 40_000] = 1.0  # N = 40000: T' = 2 of T = 16
    cases["few_nonzeros"] = x
    for name, x in cases.items():
        for threads in (1, 3, 16, 700):
            want_b = _host_nonzero_bounds(x, threads)
            want = ops.histogram_abs_chunked(x, hmax, 2048, True,
                                             torch.tensor(want_b, dtype=torch.int64, device=gpu), 0, threads)
            got = ops.histogram_abs_chunked_nonzero(x, hmax, 2048, threads)
            assert torch.equal(got, want), (name, threads)


def test_histc_skip_zeros_above_2p24_no_host_sync(gpu):
    """The calibrator's > 2^24 skip_zeros call issues no device -> host copy (the device-side
    bounds replace cumsum + int(csum[-1]) + searchsorted) and equals the per-chunk count over the
    host-computed bounds; with at most 2^24 non-zeros it equals the exact single launch."""
    from modelopt_amd import _ext
    from modelopt_amd.torch.quantization.calib.histogram import _histc_counts

    ops = _ext.ops()
    n = 2**24 + 8 * 4099
    g = torch.Generator(device=gpu).manual_seed(4)
    x = (torch.randn(n, device=gpu, generator=g)).to(torch.bfloat16)
    x[::4] = 0
    x[1::9] = 0.5
    hmax = torch.tensor([5.0], device=gpu)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        got = _histc_counts(x, hmax, 2048, True, threads=16)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    b = _host_nonzero_bounds(x, 16)
    want = ops.histogram_abs_chunked(x, hmax, 2048, True, torch.tensor(b, dtype=torch.int64, device=gpu), 0, 16)
    assert torch.equal(got, want)
    exact = torch.zeros(2048, dtype=torch.int32, device=gpu)
    ops.histogram_abs_accumulate(x, hmax, exact, 2048, True)
    assert torch.equal(got, exact.float())  # 0.75 n non-zeros < 2^24: every count exact


def test_histc_chunked_empty_input_reads_nothing(gpu):
    """an empty call of the chunked / non-zero-chunked ops (C ABI reachable) returns the
    running histogram (or zeros) without launching a count over the input."""
    from modelopt_amd import _ext

    ops = _ext.ops()
    hmax = torch.tensor([4.0], device=gpu)
    empty = torch.empty(0, dtype=torch.bfloat16, device=gpu)
    acc = torch.arange(100, dtype=torch.float32, device=gpu)
    for accum, want in ((None, torch.zeros(2048)), (acc, torch.cat([acc.cpu(), torch.zeros(1948)]))):
        got = ops.histogram_abs_chunked_nonzero(empty, hmax, 2048, 16, None, accum)
        assert torch.equal(got.cpu(), want)
        bounds = torch.zeros(17, dtype=torch.int64, device=gpu)
        got = ops.histogram_abs_chunked(empty, hmax, 2048, True, bounds, 0, 16, None, accum)
        assert torch.equal(got.cpu(), want)
