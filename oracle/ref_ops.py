"""CPU restatement of the reference's fake-quant / calibration arithmetic -- TEST INFRASTRUCTURE.

This module is the *oracle*: an independent CPU restatement of the algorithms of
``modelopt.torch.quantization`` (reference at /root/reference, cited file:line relative to its
root) that the HIP path is checked against.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker / the timed CPU
baseline -- the product (``modelopt_amd``) never imports or calls anything here.

The INT, FP8, amax and histogram restatements issue the same ATen op sequence as the reference's
eager path, so they double as the "reference CPU path" baseline timed by bench.py.  The MX
restatement follows the reference's table walk (tensor_quant_mx.h) with torch.searchsorted
rather than the minifloat arithmetic the HIP kernel uses, so the two are independent derivations.

Pinning: every function here is checked against golden vectors produced by running the
reference itself in the survey container (tests/golden/make_golden.py -> tests/golden/*.safetensors,
tests/test_oracle_golden.py) and, for the MX formats (no CPU path in the reference), against the
known-answer tables of tests/gpu/torch/quantization/test_quantize_mxformats_cuda.py:61-317
(copied as data into tests/golden/mx_kat.json).
"""

from __future__ import annotations

import math
from collections import Counter

import numpy as np
import torch

EPS = 1.0 / (1 << 24)

# ----------------------------------------------------------------------------------------------
# INT-n fake quant: restates `_tensor_quant`, modelopt/torch/quantization/tensor_quant.py:607-645
# ----------------------------------------------------------------------------------------------


def tensor_quant(inputs, amax, num_bits=8, unsigned=False, narrow_range=True):
    if unsigned and inputs.min() < 0.0:
        raise TypeError("Negative values encountered in unsigned quantization.")
    input_dtype = inputs.dtype
    inputs = inputs.float()
    amax = amax.float()
    min_amax = amax.min()
    if min_amax < 0:
        raise ValueError("Negative values in amax")
    max_bound = torch.tensor((2.0 ** (num_bits - 1 + int(unsigned))) - 1.0, device=amax.device)
    if unsigned:
        min_bound = 0
    elif narrow_range:
        min_bound = -max_bound
    else:
        min_bound = -max_bound - 1
    scale = max_bound / amax
    if min_amax <= EPS:
        zero_amax_mask = amax <= EPS
        scale[zero_amax_mask] = 0
    outputs = torch.clamp((inputs * scale).round_(), min_bound, max_bound)
    if min_amax <= EPS:
        scale[zero_amax_mask] = 1.0
    outputs = outputs / scale
    return outputs.to(input_dtype)


# ----------------------------------------------------------------------------------------------
# FP8 e4m3: restates `_fp8_eager`, tensor_quant.py:46-59
# ----------------------------------------------------------------------------------------------


def fp8_eager(x, amax=None):
    dtype = x.dtype
    if amax is not None:
        amax = amax.to(torch.float32)
        zero_amax_mask = amax <= EPS
        safe_amax = torch.where(zero_amax_mask, torch.ones_like(amax), amax)
        scale = 448.0 / safe_amax
        scale_inv = 1 / scale
        x = (x.to(torch.float32) * scale).clamp(min=-448.0, max=448.0)
    x = x.to(torch.float8_e4m3fn)
    if amax is not None:
        x = x.to(torch.float32) * scale_inv
    return x.to(dtype)


# ----------------------------------------------------------------------------------------------
# amax reductions: restates reduce_amax / convert_quantization_axis_to_reduce_axis,
# modelopt/torch/quantization/utils/core_utils.py:128-183
# ----------------------------------------------------------------------------------------------


def convert_quantization_axis_to_reduce_axis(input, axis):
    if axis is None:
        return None
    axis = axis if isinstance(axis, (list, tuple)) else [axis]
    return [i for i in range(input.dim()) if i not in axis and (i - input.dim()) not in axis]


@torch.no_grad()
def reduce_amax(input, axis=None, keepdims=True, squeeze_scalar=True):
    if input.dtype in (torch.float8_e4m3fn, torch.float8_e5m2):
        input = input.to(torch.get_default_dtype())
    if axis is None:
        max_val = torch.max(input)
        min_val = torch.min(input)
        return torch.maximum(torch.abs(max_val), torch.abs(min_val))
    if isinstance(axis, int):
        axis = (axis,)
    max_val = torch.amax(input, dim=axis, keepdim=keepdims)
    min_val = torch.amin(input, dim=axis, keepdim=keepdims)
    output = torch.maximum(torch.abs(max_val), torch.abs(min_val))
    if squeeze_scalar and output.numel() == 1:
        output.squeeze_()
    return output


class MaxCalibratorRef:
    """Restates MaxCalibrator.collect/compute_amax, calib/max.py:52-86."""

    def __init__(self, axis=None):
        self._axis = axis
        self._calib_amax = None

    def collect(self, x):
        reduce_axis = convert_quantization_axis_to_reduce_axis(x, self._axis)
        local_amax = reduce_amax(x, axis=reduce_axis).detach()
        assert not torch.any(torch.isnan(local_amax))
        assert torch.all(local_amax >= 0)
        assert not torch.any(torch.isinf(local_amax))
        if self._calib_amax is None:
            self._calib_amax = local_amax
        else:
            if local_amax.shape != self._calib_amax.shape:
                raise RuntimeError("amax shape changed!")
            self._calib_amax = torch.max(self._calib_amax, local_amax)

    def compute_amax(self):
        return self._calib_amax


# ----------------------------------------------------------------------------------------------
# Histogram calibration: restates HistogramCalibrator, calib/histogram.py:77-343
# ----------------------------------------------------------------------------------------------


class HistogramCalibratorRef:
    def __init__(self, num_bits=8, unsigned=False, num_bins=2048, skip_zeros=False):
        self._num_bits = num_bits
        self._unsigned = unsigned
        self._num_bins = num_bins
        self._skip_zeros = skip_zeros
        self._calib_bin_edges = None
        self._calib_hist = None

    def collect(self, x):
        if torch.min(x) < 0.0:
            x = x.abs()
        x = x.float()
        with torch.no_grad():
            if self._skip_zeros:
                x = x[torch.where(x != 0)]
            x_max = x.max()
            if self._calib_bin_edges is None and self._calib_hist is None:
                self._calib_hist = torch.histc(x, bins=self._num_bins, min=0, max=x_max)
                self._calib_bin_edges = torch.linspace(0, x_max, self._num_bins + 1)
            else:
                if x_max > self._calib_bin_edges[-1]:
                    width = self._calib_bin_edges[1] - self._calib_bin_edges[0]
                    self._num_bins = int((x_max / width).ceil().item())
                    self._calib_bin_edges = torch.arange(0, x_max + width, width, device=x.device)
                hist = torch.histc(x, bins=self._num_bins, min=0, max=self._calib_bin_edges[-1])
                hist[: self._calib_hist.numel()] += self._calib_hist
                self._calib_hist = hist

    def compute_amax(self, method, *, stride=1, start_bin=128, percentile=99.99):
        calib_hist = self._calib_hist.int().cpu().numpy()
        calib_bin_edges = self._calib_bin_edges.cpu().numpy()
        if method == "entropy":
            return compute_amax_entropy(
                calib_hist, calib_bin_edges, self._num_bits, self._unsigned, stride, start_bin
            )
        if method == "mse":
            return compute_amax_mse(
                calib_hist, calib_bin_edges, self._num_bits, self._unsigned, stride, start_bin
            )
        if method == "percentile":
            return compute_amax_percentile(calib_hist, calib_bin_edges, percentile)
        raise TypeError(f"Unknown calibration method {method}")


def compute_amax_entropy(calib_hist, calib_bin_edges, num_bits, unsigned, stride=1, start_bin=128):
    """Restates _compute_amax_entropy, calib/histogram.py:210-282 (loop form)."""
    from scipy.stats import entropy

    bins = calib_hist[:]
    bins[0] = bins[1]
    total_data = np.sum(bins)
    divergences = []
    nbins = 1 << (num_bits - 1 + int(unsigned))
    new_density_counts = np.zeros(nbins, dtype=np.float64)
    for i in range(start_bin, len(bins) + 1, stride):
        new_density_counts.fill(0)
        space = np.linspace(0, i, num=nbins + 1)
        digitized_space = np.digitize(range(i), space) - 1
        digitized_space[bins[:i] == 0] = -1
        for idx, digitized in enumerate(digitized_space):
            if digitized != -1:
                new_density_counts[digitized] += bins[idx]
        counter = Counter(digitized_space)
        for key, val in counter.items():
            if key != -1:
                new_density_counts[key] = new_density_counts[key] / val
        new_density = np.zeros(i, dtype=np.float64)
        for idx, digitized in enumerate(digitized_space):
            if digitized != -1:
                new_density[idx] = new_density_counts[digitized]
        total_counts_new = np.sum(new_density) + np.sum(bins[i:])
        # the reference's _normalize_distr rebinds its local and is a no-op (histogram.py:216-219);
        # scipy's entropy normalises both densities itself
        reference_density = np.array(bins[: len(digitized_space)])
        reference_density[-1] += np.sum(bins[i:])
        total_counts_old = np.sum(reference_density)
        if round(total_counts_new) != total_data or round(total_counts_old) != total_data:
            raise RuntimeError("Count mismatch!")
        divergences.append(entropy(reference_density, new_density))
    divergences = np.array(divergences)
    last_argmin = len(divergences) - 1 - np.argmin(divergences[::-1])
    return torch.tensor(calib_bin_edges[last_argmin * stride + start_bin].item())


def compute_amax_mse(calib_hist, calib_bin_edges, num_bits, unsigned, stride=1, start_bin=128):
    """Restates _compute_amax_mse, calib/histogram.py:285-325 (CPU), with its call as it binds:
    ``fake_tensor_quant(centers, amax, num_bits, unsigned)`` puts ``num_bits`` in the ``bias`` slot
    and ``unsigned`` in ``num_bits`` (FakeTensorQuantFunction.forward, tensor_quant.py:350-394:
    ``_tensor_quant(centers - bias, amax, unsigned, False, True) + bias``), and
    ``scaled_e4m3(centers, amax, 4, 3)`` misses ``M`` (TypeError)."""
    counts = torch.from_numpy(calib_hist[:]).float()
    edges = torch.from_numpy(calib_bin_edges[:]).float()
    centers = (edges[1:] + edges[:-1]) / 2
    mses, arguments = [], []
    for i in range(start_bin, len(centers), stride):
        amax = centers[i]
        if isinstance(num_bits, int) and num_bits >= 0:
            quant_centers = tensor_quant(centers - num_bits, amax, int(unsigned), False, True) + num_bits
        elif num_bits == (4, 3):
            raise TypeError("ScaledE4M3Function.forward() missing 1 required positional argument: 'M'")
        else:
            raise TypeError("Invalid num_bits.")
        mse = ((quant_centers - centers) ** 2 * counts).mean()
        mses.append(mse)
        arguments.append(i)
    argmin = np.argmin(mses)
    return centers[arguments[argmin]]


def compute_amax_percentile(calib_hist, calib_bin_edges, percentile):
    """Restates _compute_amax_percentile, calib/histogram.py:328-343."""
    if percentile < 0 or percentile > 100:
        raise ValueError("Invalid percentile. Must be in range 0 <= percentile <= 100.")
    total = calib_hist.sum()
    cdf = np.cumsum(calib_hist / total)
    idx = np.searchsorted(cdf, percentile / 100)
    return torch.tensor(calib_bin_edges[idx].item())


# ----------------------------------------------------------------------------------------------
# MX dynamic-block quant: restates amax_and_convert_kernel (tensor_quant_mx.cu:239-294) with the
# table walk of tensor_quant_mx.h:61-188, vectorised with searchsorted.
# ----------------------------------------------------------------------------------------------

_TABLES = {
    "E2M1": ([0, 0.5, 1, 1.5, 2, 3, 4, 6], False),
    "E1M2": ([0, 0.5, 1, 1.5, 2, 2.5, 3, 3.5], False),
    "E0M3": ([0, 1, 2, 3, 4, 5, 6, 7], False),
    "E3M0": ([0, 0.25, 0.5, 1, 2, 4, 8, 16], True),
    "E3M2": (
        [0, 0.0625, 0.125, 0.1875, 0.25, 0.3125, 0.375, 0.4375, 0.5, 0.625, 0.75, 0.875, 1, 1.25,
         1.5, 1.75, 2, 2.5, 3, 3.5, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28],
        False,
    ),
    "E2M3": (
        [0, 0.125, 0.25, 0.375, 0.5, 0.625, 0.75, 0.875, 1, 1.125, 1.25, 1.375, 1.5, 1.625, 1.75,
         1.875, 2, 2.25, 2.5, 2.75, 3, 3.25, 3.5, 3.75, 4, 4.5, 5, 5.5, 6, 6.5, 7, 7.5],
        False,
    ),
}
FORMAT_MAX = {
    "E4M3": 448.0, "E5M2": 57344.0, "INT8": 127.0, "E2M1": 6.0, "E0M3": 7.0, "E3M0": 16.0,
    "E1M2": 3.5, "E3M2": 28.0, "E2M3": 7.5,
}
FORMAT_CODES = {
    "E4M3": 0, "E5M2": 1, "INT8": 2, "E0M3": 3, "E1M2": 4, "E3M0": 5, "E2M1": 6, "E3M2": 7,
    "E2M3": 8, "E8M0": 9,
}


def _table_round(x, fmt):
    """round_to_even / round_away_from_zero over value/bound tables (x >= 0, float32 tensor)."""
    values, away = _TABLES[fmt]
    vals = torch.tensor(values, dtype=torch.float32)
    # bounds are the midpoints of adjacent values (the reference's *_table_bounds arrays)
    bounds = (vals[1:] + vals[:-1]) / 2
    sat = torch.isinf(x) | torch.isnan(x)
    xc = torch.where(sat, torch.zeros_like(x), x)
    if away:
        idx = torch.searchsorted(bounds, xc, right=True)
        out = vals[idx]
    else:
        i = torch.searchsorted(bounds, xc, right=False)  # first bound >= x
        i_c = i.clamp(max=len(bounds) - 1)
        tie = (i < len(bounds)) & (xc == bounds[i_c])
        idx = torch.where(tie & (i % 2 == 1), i + 1, i)
        out = vals[idx]
    return torch.where(sat, vals[-1].expand_as(x), out)


def convert_to_types(x, fmt):
    """convert_to_types (tensor_quant_mx.h:161-188) for a float32 tensor (signed)."""
    x = x.float()
    if fmt == "E4M3":
        return torch.where(torch.isnan(x), x, x.clamp(-448, 448)).to(torch.float8_e4m3fn).float()
    if fmt == "E5M2":
        return torch.where(torch.isnan(x), x, x.clamp(-57344, 57344)).to(torch.float8_e5m2).float()
    if fmt == "INT8":
        return torch.round(x).clamp(-127, 127)
    if fmt in _TABLES:
        sign = torch.where(x < 0, -1.0, 1.0)
        return _table_round(x.abs(), fmt) * sign
    return torch.zeros_like(x)


def e8m0_scale(amax, fmt):
    """compute_scale_e8m0_NV (tensor_quant_mx.cu:104-137) + the invalid-amax rule (:139-145)."""
    amax = amax.float()
    ratio = amax / FORMAT_MAX[fmt]
    bits = ratio.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    ex = (bits >> 23) & 0xFF
    sig = bits & 0x7FFFFF
    ceil_ = (sig > 0) & (ex != 0xFE) & ~((ex == 0) & (sig <= 0x400000))
    ue = torch.where(ceil_, ex - 126, ex - 127).to(torch.float64)
    scale = torch.pow(2.0, -ue).float()
    unscale = torch.pow(2.0, ue).float()
    bad = (amax == 0) | torch.isinf(amax) | torch.isnan(amax)
    one = torch.ones_like(scale)
    return torch.where(bad, one, scale), torch.where(bad, one, unscale)


def _generic_scale(amax, fmt, scale_fmt):
    """compute_scale's general path (tensor_quant_mx.cu:147-153): fp32 emax/amax widened to
    double, 1/scale rounded to fp32 and converted to the scale format, scale = 1/inv in double."""
    emax = FORMAT_MAX[fmt]
    sc = (torch.tensor(emax, dtype=torch.float32) / amax.float()).double()
    inv = convert_to_types((1.0 / sc).float(), scale_fmt).double()
    scale, unscale = (1.0 / inv).float(), inv.float()
    bad = (amax == 0) | torch.isinf(amax) | torch.isnan(amax)
    one = torch.ones_like(scale)
    return torch.where(bad, one, scale), torch.where(bad, one, unscale)


def _global_scale(gamax, lamax, fmt, scale_fmt):
    """compute_scale_with_global (tensor_quant_mx.cu:156-183)."""
    em = torch.tensor(FORMAT_MAX[fmt], dtype=torch.float32)
    sm = FORMAT_MAX[scale_fmt]
    gamax = gamax.float()
    local_unscale = lamax.float() / em  # fp32
    two_level = sm * (em / gamax).double()  # double(fp32 ratio) * double(scale max)
    luq = convert_to_types((local_unscale.double() * two_level).float(), scale_fmt).double() / two_level
    scale, unscale = (1.0 / luq).float(), luq.float()
    bad = (lamax == 0) | torch.isinf(lamax) | torch.isnan(lamax) | (gamax == 0) | torch.isinf(gamax) | torch.isnan(gamax)
    one = torch.ones_like(scale)
    return torch.where(bad, one, scale), torch.where(bad, one, unscale)


def fused_amax_convert(x, block_size, fmt, scale_fmt="E8M0", global_amax=None):
    """Per-block (last dim) dynamic quant, zero-padded partial blocks (tensor_quant_mx.cu:240-387),
    E8M0 / generic / two-level (global amax) scales.  Per-channel global amax when x is 2-D and
    global_amax has x.size(0) elements (get_global_scaling :296-310; the reference indexes it with
    the padded element index / actual cols, i.e. the row whenever cols % block_size == 0)."""
    if block_size not in (8, 16, 32):
        raise ValueError("Blocksize for fused call must be one of {8, 16, 32}")
    dtype = x.dtype
    shape = x.shape
    xf = x.float().reshape(-1, shape[-1])
    cols = shape[-1]
    pad = (-cols) % block_size
    xp = torch.nn.functional.pad(xf, (0, pad)) if pad else xf
    blocks = xp.reshape(xp.shape[0], -1, block_size)
    amax = blocks.abs().clamp(max=torch.finfo(torch.float32).max)
    amax = torch.where(torch.isnan(amax), torch.zeros_like(amax), amax).amax(-1, keepdim=True)
    if global_amax is not None:
        g = global_amax.float().reshape(-1)
        if x.dim() == 2 and g.numel() == x.shape[0]:
            ga = g.view(-1, 1, 1).expand_as(amax)
        else:
            ga = g[0].expand_as(amax)
        scale, unscale = _global_scale(ga, amax, fmt, scale_fmt)
    elif scale_fmt == "E8M0":
        scale, unscale = e8m0_scale(amax, fmt)
    else:
        scale, unscale = _generic_scale(amax, fmt, scale_fmt)
    a = blocks.abs() * scale
    q = convert_to_types(a, fmt) * unscale
    y = torch.where(blocks < 0, -q, q)
    y = y.reshape(xp.shape)[:, :cols]
    return y.reshape(shape).to(dtype)


def nvfp4_fake_quant_block(x, global_amax, block_size=16):
    """NVFP4 dynamic two-level fake quant as the reference's primary kernel computes it
    (kernels/quantization/gemm/fp4_kernel_hopper.py:33-160 with common/nvfp4_quant.py
    fp8_quantize_scale / fp4_round_magnitude), in fp32 with correctly rounded divisions."""
    dtype, shape = x.dtype, x.shape
    xf = x.float().reshape(-1, shape[-1])
    cols = shape[-1]
    pad = (-cols) % block_size
    xp = torch.nn.functional.pad(xf, (0, pad)) if pad else xf
    blocks = xp.reshape(xp.shape[0], -1, block_size)
    gs = global_amax.float().reshape(()) / torch.tensor(6.0 * 448.0, dtype=torch.float32)
    gs = torch.where(gs > 0, gs, torch.tensor(1e-12, dtype=torch.float32))
    # tl.max (fp4_kernel_hopper.py:81) is NaN-undefined in Triton; on the hardware it lowers to
    # max.f32, which skips NaN -- restated as NaN -> 0 (parity for NaN blocks: documented, not
    # pinned by a reference output).
    ab = blocks.abs()
    bmax = torch.where(torch.isnan(ab), torch.zeros_like(ab), ab).amax(-1, keepdim=True)
    s8 = bmax / (torch.tensor(6.0, dtype=torch.float32) * gs)
    s8 = torch.minimum(s8, torch.tensor(448.0))
    q8 = s8.to(torch.float8_e4m3fn).float() * gs
    q8 = torch.where(q8 >= 1e-5, q8, torch.ones_like(q8))
    a = blocks.abs() / q8
    q = _table_round(a, "E2M1")
    r = q * q8
    y = torch.where(blocks >= 0, r, -r)
    y = y.reshape(xp.shape)[:, :cols]
    return y.reshape(shape).to(dtype)


def nvfp4_scalar_quant(x, scale):
    """nvfp4_scalar_quant (common/nvfp4_quant.py): per-block fp32 scale broadcast over x's blocks."""
    xf = x.float()
    zero = scale == 0
    safe = torch.where(zero | torch.isnan(scale) | torch.isinf(scale), torch.ones_like(scale), scale)
    a = xf.abs() / safe
    r = _table_round(a, "E2M1") * safe
    y = torch.where(xf >= 0, r, -r)
    return torch.where(zero, torch.zeros_like(y), y)


def compute_fp4_scales(amax, global_amax=None, quantize_block_scales=True, fp8_max_for_normalization=448.0):
    """compute_fp4_scales (fp4_kernel.py:217-251): amax/6, FP8-quantised (scaled_e4m3 ->
    _fp8_eager) against global_amax * (448 / fp8_max) / 6 (global = max of amax if None)."""
    scale = amax.float() / 6.0
    if quantize_block_scales:
        g = amax.float().amax() if global_amax is None else global_amax.float()
        sfq = g * (448.0 / fp8_max_for_normalization) / 6.0
        scale = fp8_eager(scale, sfq)
    return scale


def static_blockwise_fp4_fake_quant(x, amax, global_amax=None, quantize_block_scales=True,
                                    fp8_max_for_normalization=448.0):
    """Static two-level NVFP4 (kernels/quantization/gemm/fp4_kernel.py:217-316): scale = amax/6,
    FP8-quantised (scaled_e4m3 = _fp8_eager) against global_amax * (448 / fp8_max) / 6; then
    nvfp4_scalar_quant per block of x.numel() / amax.numel() elements."""
    nb = amax.numel()
    block = x.numel() // nb
    scale = compute_fp4_scales(amax, global_amax, quantize_block_scales, fp8_max_for_normalization)
    xb = x.reshape(nb, block)
    y = nvfp4_scalar_quant(xb, scale.reshape(nb, 1))
    return y.reshape(x.shape).to(x.dtype)


# ----------------------------------------------------------------------------------------------
# AWQ-lite helpers: restate model_calib.py:1453-1495
# ----------------------------------------------------------------------------------------------


def awq_weight_scale(weight, block_size=None):
    org_shape = weight.shape
    slice_after_padding = None
    if block_size:
        if org_shape[-1] % block_size != 0:
            slice_after_padding = slice(org_shape[-1])
            weight = torch.nn.functional.pad(
                weight, (0, block_size - org_shape[-1] % block_size), "constant", 0
            )
            org_shape = weight.shape
        weight = weight.contiguous().view(-1, block_size)
    weight_abs = weight.abs()
    weight_abs_amax = weight_abs.amax(dim=1, keepdim=True)
    scale = weight_abs / (weight_abs_amax + torch.finfo(weight.dtype).tiny)
    scale = scale.view(org_shape)
    if slice_after_padding is not None:
        scale = scale[..., slice_after_padding]
    return scale.mean(0).to(torch.float32)


def awq_act_scale(x):
    return x.abs().contiguous().view(-1, x.shape[-1]).mean(0).to(torch.float32)


def awq_get_scale(x_max, w_max, alpha):
    scales = (
        (x_max.pow(alpha) / (w_max.to(x_max.device).pow(1 - alpha) + torch.finfo(torch.float32).tiny))
        .clamp(min=1e-4, max=1e4)
        .view(-1)
    )
    return (scales / (scales.max() * scales.min()).sqrt()).view(-1)


def int_block_qdq_dynamic(w, block, num_bits=4, pre_quant_scale=None, unsigned=False,
                          narrow_range=False):
    """TensorQuantizer static block INT path with a dynamic amax (tensor_quantizer.py:736-751,
    :975-1061) after `inputs * pre_quant_scale` (:1143-1144)."""
    if pre_quant_scale is not None:
        w = w * pre_quant_scale
    shape = w.shape
    wb = w.reshape(-1, block)
    amax = reduce_amax(wb, axis=[1], keepdims=True)
    return tensor_quant(wb, amax, num_bits, unsigned, narrow_range).reshape(shape)


def cpu_threads() -> int:
    return torch.get_num_threads()


__all__ = [name for name in dir() if not name.startswith("_") and name not in ("math", "np", "torch")]


# ----------------------------------------------------------------------------------------------
# Checkpoint-export packing: restates export/quant_utils.py:792-938 and qtensor quantize()
# ----------------------------------------------------------------------------------------------


def export_fp8(weight, scale):
    """(weight / scale).to(float8_e4m3fn) as bytes (quant_utils.py:855-867 / :881-913)."""
    return (weight / scale).to(torch.float8_e4m3fn).view(torch.uint8)


def export_int4(weight, scale):
    """pack_int4_in_uint8 (quant_utils.py:792-833), 2-D."""
    out_dim, in_dim = weight.shape
    block = in_dim // scale.shape[-1]
    q = (weight / scale[:, torch.arange(in_dim) // block]).round().clamp(-8, 7).to(torch.int8)
    r = q.T.reshape(in_dim, out_dim // 2, 2)
    packed = (r[..., 0] & 0x0F) | ((r[..., 1] & 0x0F) << 4)
    return packed.T.contiguous().view(torch.uint8)


_NV_BOUNDS = torch.tensor([0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5])


def export_nvfp4(weight, block_scale, scale_2):
    """NVFP4QTensor.quantize with given scales (qtensor/nvfp4_tensor.py:253-342)."""
    shape = weight.shape
    block = weight.numel() // block_scale.numel()
    w = weight.reshape(*shape[:-1], -1, block)
    scaled = (w / (block_scale.float().reshape(*shape[:-1], -1) * scale_2).unsqueeze(-1)).reshape(shape)
    sign = (scaled < 0).to(torch.uint8)
    a = scaled.abs()
    ordv = torch.searchsorted(_NV_BOUNDS, a, out_int32=True).to(torch.uint8)
    eq = torch.any(a.unsqueeze(-1) == _NV_BOUNDS[[1, 3, 5]], dim=-1).to(torch.uint8)
    q = (sign << 3) + ordv + eq
    return (q[..., 1::2] << 4) | q[..., 0::2]


def export_mxfp4(weight, block=32):
    """MXFP4QTensor.quantize (qtensor/mxfp4_tensor.py:38-81): (packed codes, E8M0 bytes)."""
    shape = weight.shape
    x = weight.reshape(-1, block)
    amax = x.float().abs().max(dim=-1, keepdim=True).values
    descale = amax / 6.0
    e = torch.ceil(torch.maximum(torch.log2(descale), torch.tensor(-127.0)))
    q = (x / torch.exp2(e)).reshape(shape)
    sign_bit = (2 - torch.sign(q)) // 2
    ordv = torch.sum((q.abs().unsqueeze(-1) - _NV_BOUNDS) > 0, dim=-1)
    codes = (sign_bit * 8 + ordv).to(torch.uint8)
    packed = (codes[..., 1::2] << 4) + codes[..., 0::2]
    return packed, (e + 127).to(torch.uint8)


# ----------------------------------------------------------------------------------------------
# MSE weight calibration: calib/mse.py:31-300, model_calib.py:639-827,
# kernels/quantization/gemm/{_fp8_scale_candidates.py:25-32, nvfp4_fp8_sweep.py:62-160}
# ----------------------------------------------------------------------------------------------


def fp8_scale_candidates():
    """The 126 finite positive E4M3 values / 448 (_fp8_scale_candidates.py:25-32), fp32."""
    u = torch.arange(0, 128, dtype=torch.uint8).view(torch.float8_e4m3fn).float()
    return u[torch.isfinite(u) & (u > 0)] / 448.0


def _fp4_round_magnitude(a):
    """common/nvfp4_quant.py:31-62: nearest E2M1 magnitude by the reference's threshold chain."""
    return np.where(a <= 0.25, 0.0, np.where(a < 0.75, 0.5, np.where(a <= 1.25, 1.0, np.where(
        a < 1.75, 1.5, np.where(a <= 2.5, 2.0, np.where(a < 3.5, 3.0, np.where(a <= 5.0, 4.0, 6.0))))))).astype(np.float32)


def nvfp4_fp8_scale_sweep(x, global_amax, block_size=16):
    """Per-block best amax of the fused FP8-scale sweep (nvfp4_fp8_sweep.py:62-105): for each of the
    126 candidates c, ``scale = RN(RN(c*g)/6)`` (1 when 0), ``loss = sum((|w| - e2m1(|w|/scale)*scale)^2)``
    in fp32 with the row sum in the 8-way pairwise order of numpy (= the Triton interpreter's
    tl.sum, which the golden vectors come from), strict ``<`` so the first minimum wins, and
    ``best = RN(g * c[best])``."""
    w = np.abs(x.detach().float().reshape(-1, block_size).numpy())
    g = np.float32(float(global_amax))
    cands = fp8_scale_candidates().numpy()
    best_loss = np.full(w.shape[0], np.inf, dtype=np.float32)
    best_idx = np.zeros(w.shape[0], dtype=np.int64)
    for k, c in enumerate(cands):
        scale = np.float32(np.float32(c * g) / np.float32(6.0))
        safe = np.float32(1.0) if scale == 0 else scale
        qm = _fp4_round_magnitude((w / safe).astype(np.float32))
        diff = (w - (qm * safe).astype(np.float32)).astype(np.float32)
        loss = np.sum(diff * diff, axis=1, dtype=np.float32)
        better = loss < best_loss
        best_loss = np.where(better, loss, best_loss)
        best_idx = np.where(better, k, best_idx)
    return torch.from_numpy((g * cands[best_idx]).astype(np.float32))


def mse_candidates(step_size=0.1, start_multiplier=0.25, stop_multiplier=4.0):
    """MseCalibrator._generate_candidates (calib/mse.py:58-80)."""
    n = math.ceil((stop_multiplier - start_multiplier) / step_size) + 1
    return torch.linspace(start_multiplier, stop_multiplier, steps=n)


def mse_sweep(x, initial_amax, quant_fn, axis, candidates=None):
    """MseCalibrator.collect + compute_amax (calib/mse.py:82-183) for one tensor: per candidate
    ``xq = quant_fn(x, initial_amax * c)``, ``loss = sum((x - xq)^2)`` over the non-axis dims, then
    the first argmin per channel.  Returns (losses [K, ...], best amax)."""
    x = x.detach().float()
    cands = mse_candidates() if candidates is None else candidates
    red = convert_quantization_axis_to_reduce_axis(x, axis)
    losses = []
    for c in cands:
        xq = quant_fn(x, initial_amax * c)
        err = torch.nn.functional.mse_loss(x, xq, reduction="none")
        losses.append(torch.sum(err) if red is None else torch.sum(err, dim=red))
    losses = torch.stack(losses)
    best = cands[torch.argmin(losses, dim=0)]
    if best.ndim != 0:
        best = best.view_as(initial_amax)
    return losses, initial_amax * best


# ----------------------------------------------------------------------------------------------
# AWQ-clip block search: model_calib.py:1725-1940 (_clip_search :1800-1882, update_best_params
# :1785-1797)
# ----------------------------------------------------------------------------------------------


def awq_clip_shrinks(min_clip_ratio=0.5, shrink_step=0.05):
    """model_calib.py:1757-1759."""
    return [round(float(k), 2) for k in torch.arange(min_clip_ratio, 1.0, shrink_step)] + [1.0]


def awq_clip_block_losses(weight, inputs, w_amax, shrinks, block, num_bits=4, unsigned=False,
                          narrow_range=False, co_bsz=1024, max_tokens=64):
    """One `_clip_search` call (model_calib.py:1815-1882) for a static-block INT-n weight: returns
    ({shrink: loss [co_batch rows, n_block]} stacked as [S, co, n_block], tokens used).  The ATen
    op sequence is the reference's: stride-sampled tokens, zero padding to the block, the
    dtype-rounded ``(inputs * w).sum(-1)`` per block, ``(cur - org).float().pow(2).mean(1)``."""
    co, ci = weight.shape
    x = inputs.reshape(-1, inputs.shape[-1])
    x = x[0 :: max(1, x.shape[0] // max_tokens)]
    ntok = x.shape[0]
    w = weight
    if ci % block:
        w = torch.nn.functional.pad(w, (0, block - ci % block), "constant", 0)
        x = torch.nn.functional.pad(x, (0, block - ci % block), "constant", 0)
    cip = w.shape[-1]
    w4 = w.reshape(co, 1, -1, block)
    x4 = x.reshape(1, ntok, -1, block)
    out = torch.zeros(len(shrinks), co, cip // block)
    for s_i, shrink in enumerate(shrinks):
        amax = w_amax * shrink
        # the weight quantizer's static block path: blocks of the (padded) weight, per-block amax
        wq = tensor_quant(w.reshape(-1, block), amax.reshape(-1, 1), num_bits, unsigned, narrow_range)
        wq = wq.reshape(co, 1, -1, block)
        for b0 in range(0, co, co_bsz):
            sl = slice(b0, min(b0 + co_bsz, co))
            org = (x4 * w4[sl]).sum(dim=-1)
            cur = (x4 * wq[sl]).sum(dim=-1)
            out[s_i, sl] = (cur - org).float().pow(2).mean(dim=1)
    return out, ntok


def awq_clip_best(losses, w_amax, shrinks):
    """update_best_params (model_calib.py:1785-1797): first strictly-smaller loss wins."""
    best_loss = torch.ones_like(w_amax) * float("inf")
    best = torch.zeros_like(w_amax)
    for s_i, shrink in enumerate(shrinks):
        loss = losses[s_i].reshape(w_amax.shape)
        idx = loss < best_loss
        best_loss = torch.where(idx, loss, best_loss)
        best = torch.where(idx, w_amax * shrink, best)
    return best


# ----------------------------------------------------------------------------------------------
# MXFP8 (E4M3 elements, E8M0 scale per 32): restates MXFP8QTensor._compute_e8m0_exponent +
# quantize_with_scale, quantization/qtensor/mxfp8_tensor.py:36-52, 140-187
# ----------------------------------------------------------------------------------------------


def mxfp8_quantize(weight, block=32):
    """(e4m3 codes as float8_e4m3fn, E8M0 bytes [..., K/32]) of a [..., K] weight, K % 32 == 0."""
    shape = weight.shape
    blocks = weight.reshape(*shape[:-1], shape[-1] // block, block)
    amax = blocks.abs().amax(dim=-1)
    descale = amax.float() / 448.0
    log2 = torch.where(descale > 0, torch.log2(descale), torch.tensor(-127.0))
    e = torch.clamp(torch.ceil(log2), min=-127, max=127)
    s = (e + 127).to(torch.uint8)
    f = torch.exp2(127 - s.float()).unsqueeze(-1)
    q = (blocks * f).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).reshape(shape)
    return q, s
