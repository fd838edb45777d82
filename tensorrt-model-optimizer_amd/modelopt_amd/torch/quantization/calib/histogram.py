"""Histogram calibrator on the LDS-privatised |x| histogram kernel.

Reference: modelopt/torch/quantization/calib/histogram.py:35-343.  ``collect`` keeps the
reference's torch-histogram branch semantics exactly (``torch.histc(|x|, bins, 0, max)`` with the
first-call ``linspace`` edges and the fixed-width bin growth of :108-130); the histogram itself is
one launch of ``histogram_abs_accumulate`` plus one of the max|x| reduction (the reference: abs,
float copy, max, histc -- and a ``torch.min(x) < 0`` host sync).

Counts follow ``torch.histc``'s float semantics (``_histc_counts``): the reference's CPU histc
splits the (flattened, after ``skip_zeros``) input into one contiguous chunk per intra-op thread,
counts each chunk into a thread-local fp32 histogram -- a count stops at 2^24, where ``+1`` rounds
back to 2^24 -- and adds the per-thread histograms in thread order in fp32 (measured on torch
2.10: chunk counts (2^24+, 3, 3) give 16777224, (3, 3, 2^24+) give 16777222).  The kernel counts
exact integers per chunk; when a call can hold more than 2^24 elements, the chunks are counted
separately and folded exactly so, with the calibrator's recorded thread count
``_histc_threads``: fixed at its first ``collect`` from ``torch.get_num_threads()`` (the
reference's own process setting; ``MTQ_AMD_HIST_THREADS`` overrides) and saved with the quantizer
state, so a restored calibrator counts exactly as the one that recorded it whatever the new
process's ``OMP_NUM_THREADS`` (a torchrun launch sets 1).  ``MTQ_AMD_HIST_COUNTS=exact`` keeps
exact integer counts instead.

``compute_amax`` runs on the host like the reference (entropy / MSE / percentile).  The MSE sweep
reproduces the reference's actual call ``fake_tensor_quant(centers, amax, num_bits, unsigned)``,
which binds ``num_bits`` to the functional's ``bias`` slot and ``unsigned`` to ``num_bits``
(histogram.py:305-312 vs tensor_quant.py:349-391); ``MTQ_AMD_HIST_MSE=intent`` quantises with the
documented intent instead (``num_bits``-bit, no bias).
"""

from __future__ import annotations

import os
import warnings
from collections import Counter

import numpy as np
import torch

from modelopt_amd._ext import ops as _ops

from ..tensor_quant import fake_tensor_quant, fp8_fake_quant
from ..utils import core_utils as quant_utils
from .calibrator import _Calibrator

__all__ = ["HistogramCalibrator"]


class HistogramCalibrator(_Calibrator):
    def __init__(
        self,
        num_bits=8,
        axis=None,
        unsigned=False,
        num_bins=2048,
        grow_method=None,
        skip_zeros=False,
        torch_hist=True,
    ):
        super().__init__(num_bits, axis, unsigned)
        self._num_bins = num_bins
        self._skip_zeros = skip_zeros
        self._calib_bin_edges = None
        self._calib_hist = None
        self._torch_hist = torch_hist
        # chunk count of the >2^24-element histc emulation, recorded at the first collect
        self._histc_threads = None
        if axis is not None:
            raise NotImplementedError("Calibrator histogram collection only supports per tensor scaling")
        if not torch_hist:
            raise NotImplementedError(
                "modelopt_amd: the numpy (host) histogram branch is not part of the MI355X path; "
                "use torch_hist=True"
            )

    @torch.no_grad()
    def collect(self, x):
        if x.dtype not in (torch.float32, torch.float16, torch.bfloat16):
            x = x.float()  # the reference histograms x.float() (histogram.py:82); exact for ints
        if self._histc_threads is None:
            self._histc_threads = _histc_threads()
        # max|x| (equals the reference's max over the non-zero |x| when skip_zeros, histogram.py:105-112)
        x_max = torch.zeros((), dtype=torch.float32, device=x.device)
        quant_utils.reduce_amax_accumulate(x, x_max, None)
        if self._calib_bin_edges is None and self._calib_hist is None:
            hmax = x_max
            bins = self._num_bins
            self._calib_bin_edges = torch.linspace(0, float(x_max), self._num_bins + 1)
            old = None
        else:
            xm = x_max.cpu()
            if float(xm) > float(self._calib_bin_edges[-1]):
                width = (self._calib_bin_edges[1] - self._calib_bin_edges[0]).cpu()
                self._num_bins = int((xm / width).ceil().item())
                # the edges are host bookkeeping: built with the CPU arange (double accumulation),
                # the reference-CPU semantics; a device arange rounds the edges differently
                self._calib_bin_edges = torch.arange(0, xm + width, width)
            bins = self._num_bins
            hmax = self._calib_bin_edges[-1].to(device=x.device, dtype=torch.float32).reshape(())
            old = self._calib_hist
        if old is not None:
            old = old.to(x.device)
        self._calib_hist = _histc_counts(x, hmax.float().contiguous(), bins, self._skip_zeros,
                                         self._histc_threads, accum=old)

    def reset(self):
        self._calib_bin_edges = None
        self._calib_hist = None

    def compute_amax(self, method: str, *, stride: int = 1, start_bin: int = 128, percentile: float = 99.99):
        import torch.distributed as tdist

        if tdist.is_available() and tdist.is_initialized():
            warnings.warn(
                "This method does not perform any synchronization across distributed processes. The "
                "recommended method is to use the same calibration dataset across all distributed data "
                "parallel groups so that `amax` is the same for all DDP modules."
            )
        if self._calib_hist is None:
            return None
        calib_hist = self._calib_hist.int().cpu().numpy()
        calib_bin_edges = self._calib_bin_edges.cpu().numpy()
        if method == "entropy":
            return _compute_amax_entropy(
                calib_hist, calib_bin_edges, self._num_bits, self._unsigned, stride, start_bin
            )
        if method == "mse":
            return _compute_amax_mse(
                calib_hist, calib_bin_edges, self._num_bits, self._unsigned, stride, start_bin,
                device=self._calib_hist.device,
            )
        if method == "percentile":
            return _compute_amax_percentile(calib_hist, calib_bin_edges, percentile)
        raise TypeError(f"Unknown calibration method {method}")

    def __str__(self):
        if self._calib_bin_edges is None:
            e = "None"
        else:
            e = f"[{float(self._calib_bin_edges[0]):.3f}, ..., {float(self._calib_bin_edges[-1]):.3f}]({len(self._calib_bin_edges)})"
        return f"HistogramCalibrator(calib_bin_edges={e})"


_HISTC_GRAIN = 32768  # at::internal::GRAIN_SIZE: the parallel_for grain of the CPU histc
_F32_COUNT_LIMIT = 2**24  # an fp32 counter stops here: 2^24 + 1 rounds to 2^24 (ties to even)


def _histc_threads() -> int:
    env = os.environ.get("MTQ_AMD_HIST_THREADS")
    return max(1, int(env)) if env else max(1, torch.get_num_threads())


# the one-read skip_zeros path (csrc/mtq_kernels.hip mtq_histogram_abs_nonzero_chunked) takes up to
# ~6e10 elements; larger calls take the per-chunk path
_NZ_ONE_READ_MAX_ELEMS = 50_000_000_000


def _histc_counts(x: torch.Tensor, hmax: torch.Tensor, bins: int, skip_zeros: bool,
                  threads: int | None = None, accum: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 per-call histogram of |x| over [0, hmax] with torch.histc's CPU accumulation.

    Every count of a call with at most 2^24 (kept) elements is exact in fp32 whatever the chunking,
    so one launch does.  Above that, the chunk of thread t of at::parallel_for (``T = threads``,
    default ``_histc_threads()``; chunk = ceil(N / T), N = elements after ``skip_zeros``) is counted
    exactly, clamped at 2^24 and added into the fp32 result in thread order: bf16 / f16 on the GPU
    in one counting launch for all chunks plus one fold launch (histogram_abs_chunked; with
    ``skip_zeros`` the non-zero chunk boundaries are found on the device first,
    histogram_abs_chunked_nonzero), other inputs one launch per chunk.  ``accum`` (the
    calibrator's running histogram, ``numel <= bins``) is added into the first bins of the result
    (``hist[:old.numel()] += old``, reference histogram.py:127), in the fold launch on the GPU
    path."""

    def plus_accum(hist):
        if accum is not None:
            hist[: accum.numel()] += accum
        return hist

    ops = _ops()
    n = x.numel()
    mode = os.environ.get("MTQ_AMD_HIST_COUNTS", "histc")
    if n <= _F32_COUNT_LIMIT or mode == "exact":
        counts = torch.zeros(bins, dtype=torch.int32, device=x.device)
        ops.histogram_abs_accumulate(x, hmax, counts, bins, skip_zeros)
        return plus_accum(counts.float())
    flat = x.contiguous().reshape(-1)
    gpu_one_launch = (flat.is_cuda and flat.dtype in (torch.bfloat16, torch.float16) and bins <= 8192
                      and n % 8 == 0 and flat.data_ptr() % 16 == 0)
    t = threads or _histc_threads()
    if skip_zeros and gpu_one_launch and bins <= 8176 and t <= 1024 and n <= _NZ_ONE_READ_MAX_ELEMS:
        # the non-zero chunks counted on the device in one read of the input, no host sync (the
        # boundaries resolved afterwards from per-slab non-zero counts); with at most 2^24
        # non-zeros every count is exact in fp32, so the chunked sum equals the single-launch count
        return ops.histogram_abs_chunked_nonzero(flat, hmax, bins, t, None, accum)
    if skip_zeros:
        # chunk boundaries live in the compacted (non-zero) index space: map them back
        csum = torch.cumsum((flat != 0).to(torch.int64), 0)
        kept = int(csum[-1])
    else:
        csum, kept = None, n
    if kept <= _F32_COUNT_LIMIT:
        counts = torch.zeros(bins, dtype=torch.int32, device=x.device)
        ops.histogram_abs_accumulate(flat, hmax, counts, bins, skip_zeros)
        return plus_accum(counts.float())
    threads = min(threads or _histc_threads(), -(-kept // _HISTC_GRAIN))
    chunk = -(-kept // threads)
    starts = [t * chunk for t in range(threads) if t * chunk < kept] + [kept]
    cuts = None
    if csum is not None:
        # the first original index whose non-zero rank reaches each compacted start
        cuts = torch.searchsorted(csum, torch.tensor(starts[1:-1], device=csum.device, dtype=torch.int64) + 1)
    if gpu_one_launch:
        # one launch counts every chunk (per-workgroup rows), a second adds the clamped chunk
        # counts in order (scratch: the caching allocator's, any contents)
        nch = len(starts) - 1
        return ops.histogram_abs_chunked(flat, hmax, bins, False, None, chunk, nch, None, accum)
    bounds = [0] + cuts.tolist() + [n] if cuts is not None else starts
    hist = torch.zeros(bins, dtype=torch.float32, device=x.device)
    counts = torch.empty(bins, dtype=torch.int32, device=x.device)
    for b, e in zip(bounds[:-1], bounds[1:]):
        counts.zero_()
        if e > b:
            ops.histogram_abs_accumulate(flat[b:e], hmax, counts, bins, skip_zeros)
        hist += counts.float().clamp_(max=_F32_COUNT_LIMIT)
    return plus_accum(hist)


def _compute_amax_entropy(calib_hist, calib_bin_edges, num_bits, unsigned, stride=1, start_bin=128):
    """KL-divergence amax (histogram.py:210-282).

    Same arithmetic as the reference loop, with the per-candidate Python loops replaced by numpy
    gathers/bincounts: for candidate i the quantised density assigns every non-empty bin j < i the
    mean count of the non-empty bins in its quantisation level (np.digitize over linspace(0, i)).
    """
    from scipy.stats import entropy

    if calib_bin_edges is None and calib_hist is None:
        return None
    bins = calib_hist[:]
    bins[0] = bins[1]
    total_data = np.sum(bins)
    divergences = []
    nbins = 1 << (num_bits - 1 + int(unsigned))
    for i in range(start_bin, len(bins) + 1, stride):
        space = np.linspace(0, i, num=nbins + 1)
        digitized = np.digitize(range(i), space) - 1
        digitized[bins[:i] == 0] = -1
        valid = digitized != -1
        dv = digitized[valid]
        level_sum = np.zeros(nbins, dtype=np.float64)
        # sequential accumulation order matters for float64 sums of integers < 2^53: exact anyway
        np.add.at(level_sum, dv, bins[:i][valid].astype(np.float64))
        level_cnt = np.bincount(dv, minlength=nbins)
        with np.errstate(invalid="ignore", divide="ignore"):
            level_mean = np.where(level_cnt > 0, level_sum / np.maximum(level_cnt, 1), 0.0)
        new_density = np.zeros(i, dtype=np.float64)
        new_density[valid] = level_mean[dv]
        total_counts_new = np.sum(new_density) + np.sum(bins[i:])
        # the reference's _normalize_distr rebinds its local and is a no-op (histogram.py:216-219);
        # scipy's entropy normalises both densities itself
        reference_density = np.array(bins[: len(digitized)])
        reference_density[-1] += np.sum(bins[i:])
        total_counts_old = np.sum(reference_density)
        if round(total_counts_new) != total_data or round(total_counts_old) != total_data:
            raise RuntimeError(
                f"Count mismatch! total_counts_new={total_counts_new}, "
                f"total_counts_old={total_counts_old}, total_data={total_data}"
            )
        divergences.append(entropy(reference_density, new_density))
    divergences = np.array(divergences)
    last_argmin = len(divergences) - 1 - np.argmin(divergences[::-1])
    return torch.tensor(calib_bin_edges[last_argmin * stride + start_bin].item())


def _reference_call_qdq(centers: torch.Tensor, amax: torch.Tensor, bias: int, num_bits: int) -> torch.Tensor:
    """What the reference's ``fake_tensor_quant(centers, amax, num_bits, unsigned)`` computes on
    the CPU (histogram.py:308): ``bias = num_bits`` and ``num_bits = unsigned`` (0 or 1), so
    FakeTensorQuantFunction.forward (tensor_quant.py:350-394) quantises ``centers - bias`` with
    ``_tensor_quant(..., num_bits, unsigned=False, narrow_range=True)`` (:607-645) and adds the
    bias back -- the same fp32 operations, elementwise, in the same order."""
    x = (centers - bias).float()
    a = amax.float()
    max_bound = torch.tensor(2.0 ** (num_bits - 1) - 1.0, dtype=torch.float32)
    min_bound = -max_bound
    scale = max_bound / a
    tiny = bool(a <= 1.0 / (1 << 24))
    if tiny:
        scale = torch.zeros_like(scale)
    out = torch.clamp((x * scale).round_(), min_bound, max_bound)
    if tiny:
        scale = torch.ones_like(scale)
    return (out / scale) + bias


_warned_mse = [False]


def _compute_amax_mse(calib_hist, calib_bin_edges, num_bits, unsigned, stride=1, start_bin=128,
                      device=None):
    """MSE amax (histogram.py:285-325).

    Default: the reference's actual numbers.  Its call ``fake_tensor_quant(centers, amax, num_bits,
    unsigned)`` binds ``num_bits`` to ``bias`` (``_reference_call_qdq``), and ``scaled_e4m3(centers,
    amax, 4, 3)`` lacks ``M`` and raises TypeError -- both reproduced.  The sweep runs on the host
    in fp32 with the reference's per-candidate op sequence (2048 bins, once per quantizer), so the
    chosen amax is the reference run's bit for bit (``tests/golden/calib_ref.*``); the reference
    itself moves it to the GPU when one is present, where its CUDA extension evaluates the
    0-bit shift of the same call differently (tensor_quant_gpu.cu:38-41) -- parity is pinned to
    the CPU run.  ``MTQ_AMD_HIST_MSE=intent``: quantise with ``num_bits`` bits (narrow range) and
    FP8 E4M3 as the code evidently intends, on the calibrator's device with the HIP kernels.
    """
    if calib_bin_edges is None and calib_hist is None:
        return None
    intent = os.environ.get("MTQ_AMD_HIST_MSE", "reference") == "intent"
    if not intent and not _warned_mse[0]:
        _warned_mse[0] = True
        warnings.warn(
            "HistogramCalibrator 'mse': reproducing the reference's actual candidate quantisation "
            "(fake_tensor_quant(centers, amax, num_bits, unsigned) binds num_bits to `bias` and "
            "unsigned to `num_bits`; FP8 raises TypeError) for parity; MTQ_AMD_HIST_MSE=intent "
            "quantises the candidates with num_bits bits / E4M3 instead.",
            stacklevel=3,
        )
    counts = torch.from_numpy(calib_hist[:]).float()
    edges = torch.from_numpy(calib_bin_edges[:]).float()
    if intent and device is not None and device.type == "cuda":
        counts = counts.to(device)
        edges = edges.to(device)
    centers = (edges[1:] + edges[:-1]) / 2
    mses, arguments = [], []
    for i in range(start_bin, len(centers), stride):
        amax = centers[i]
        if isinstance(num_bits, int) and num_bits >= 0:
            if intent:
                quant_centers = fake_tensor_quant(centers, amax, None, num_bits, unsigned)
            else:
                quant_centers = _reference_call_qdq(centers, amax, num_bits, int(unsigned))
        elif num_bits == (4, 3):
            if not intent:
                raise TypeError("ScaledE4M3Function.forward() missing 1 required positional argument: 'M'")
            quant_centers = fp8_fake_quant(centers, amax)
        else:
            raise TypeError("Invalid num_bits. num_bits must be a positive integer or tuple (4,3).")
        mses.append(((quant_centers - centers) ** 2 * counts).mean())
        arguments.append(i)
    mses_np = torch.stack(mses).cpu().numpy()
    argmin = np.argmin(mses_np)
    calib_amax = centers[arguments[argmin]]
    if device is not None:
        calib_amax = calib_amax.to(device)
    return calib_amax


def _compute_amax_percentile(calib_hist, calib_bin_edges, percentile):
    """Percentile amax (histogram.py:328-343)."""
    if percentile < 0 or percentile > 100:
        raise ValueError("Invalid percentile. Must be in range 0 <= percentile <= 100.")
    if calib_bin_edges is None and calib_hist is None:
        return None
    total = calib_hist.sum()
    cdf = np.cumsum(calib_hist / total)
    idx = np.searchsorted(cdf, percentile / 100)
    return torch.tensor(calib_bin_edges[idx].item())


_ = Counter  # kept for parity with the reference module's imports
