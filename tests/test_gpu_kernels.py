"""HIP kernels (through the torch ops over the C ABI) vs the CPU oracle, bit for bit.

Mirrors the reference's two-oracle pattern (tests/gpu/torch/quantization/test_tensor_quant_cuda.py:
ext == ATen path bit-exact for INT, FP8 ext == fp8_eager): here HIP == oracle/ref_ops.py, and the
oracle itself is pinned to the reference by tests/test_oracle_golden.py.
"""

import math

import pytest
import torch

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu

DTYPES = [torch.float32, torch.float16, torch.bfloat16]


def same_bits(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Bitwise equality, NaN == NaN (any payload); -0 vs +0 distinguished."""
    a = a.detach().cpu()
    b = b.detach().cpu()
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    nan = torch.isnan(a.float()) & torch.isnan(b.float())
    if a.dtype == torch.float64:
        ia, ib = a.view(torch.int64), b.view(torch.int64)
    elif a.dtype == torch.float32:
        ia, ib = a.view(torch.int32), b.view(torch.int32)
    else:
        ia, ib = a.view(torch.int16), b.view(torch.int16)
    return bool(((ia == ib) | nan).all())


def mismatch(a, b):
    a = a.detach().cpu().float()
    b = b.detach().cpu().float()
    bad = ~((a == b) | (torch.isnan(a) & torch.isnan(b)))
    idx = bad.nonzero()[:5]
    return f"{int(bad.sum())} mismatches, e.g. at {idx.tolist()}: {a[bad][:5].tolist()} vs {b[bad][:5].tolist()}"


def rand_with_edges(shape, dtype, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(shape, generator=g) * scale
    flat = x.view(-1)
    n = flat.numel()
    # half-way points for rounding ties, signed zeros, big outliers
    k = max(1, n // 64)
    flat[:k] = torch.round(flat[:k] * 8) / 8 + 0.5 / 8
    flat[k : 2 * k] = 0.0
    flat[2 * k : 3 * k] = -0.0
    flat[3 * k] = 7.5 * scale
    return x.to(dtype)


def ops():
    from modelopt_amd import _ext

    return _ext.ops()


# --------------------------------------------------------------------------------------------
# INT
# --------------------------------------------------------------------------------------------


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("num_bits", [3, 4, 5, 7, 8, 11])
@pytest.mark.parametrize("unsigned,narrow", [(False, True), (False, False), (True, False)])
def test_int_per_tensor(gpu, dtype, num_bits, unsigned, narrow):
    x = rand_with_edges((37, 129), dtype, seed=num_bits)
    if unsigned:
        x = x.abs()
    amax = x.float().abs().amax() * 0.7
    ref = R.tensor_quant(x, amax, num_bits, unsigned, narrow)
    out = ops().fake_tensor_quant(x.to(gpu), amax.to(gpu), num_bits, unsigned, narrow)
    assert same_bits(out, ref), mismatch(out, ref)


@pytest.mark.parametrize("dtype", DTYPES)
def test_int_vectorised_and_tail(gpu, dtype):
    # large enough for the unrolled vector loop, odd length for the scalar tail
    x = rand_with_edges((1 << 20) + 3, dtype, seed=5)
    amax = torch.tensor(2.5)
    ref = R.tensor_quant(x, amax, 8, False, False)
    out = ops().fake_tensor_quant(x.to(gpu), amax.to(gpu), 8, False, False)
    assert same_bits(out, ref), mismatch(out, ref)
    # unaligned view (offset by one element) takes the scalar path
    xs = x[1:]
    out = ops().fake_tensor_quant(x.to(gpu)[1:], amax.to(gpu), 8, False, False)
    ref = R.tensor_quant(xs, amax, 8, False, False)
    assert same_bits(out, ref), mismatch(out, ref)


@pytest.mark.parametrize("amax_val", [0.0, 2.0**-24, 2.0**-25, 1e-30])
def test_int_zero_amax(gpu, amax_val):
    x = torch.tensor([1.0, -1.0, 0.0, -0.0, float("nan"), float("inf")], dtype=torch.float32)
    amax = torch.tensor(amax_val)
    ref = R.tensor_quant(x, amax, 8)
    out = ops().fake_tensor_quant(x.to(gpu), amax.to(gpu), 8, False, True)
    assert same_bits(out, ref), mismatch(out, ref)


def test_int_special_values(gpu):
    x = torch.tensor([float("nan"), float("inf"), -float("inf"), 1e30, -1e30, 0.0, -0.0, 3.5, -3.5])
    amax = torch.tensor(7.0)
    ref = R.tensor_quant(x, amax, 4, False, False)
    out = ops().fake_tensor_quant(x.to(gpu), amax.to(gpu), 4, False, False)
    assert same_bits(out, ref), mismatch(out, ref)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize(
    "shape,amax_shape",
    [
        ((64, 256), (64, 1)),  # per-row (weight axis 0)
        ((64, 256), (1, 256)),  # per-column (axis -1): element-wise channel path
        ((4, 6, 40), (1, 6, 1)),  # middle axis
        ((4, 6, 40), (4, 6, 1)),  # merged leading axes (per-token)
        ((4096, 128), (4096, 1)),  # block-128 view of a weight
        ((33, 24), (33, 1)),  # inner 24 = 3 bf16 vectors
        ((16, 2048), (16, 1)),  # long rows: wave-uniform channel kernel (ew_rowwave_kernel)
        ((6, 1024), (6, 1)),  # long rows, 128 bf16 vectors each (the kernel's minimum)
    ],
)
def test_int_axis(gpu, dtype, shape, amax_shape):
    x = rand_with_edges(shape, dtype, seed=11)
    g = torch.Generator().manual_seed(3)
    amax = torch.rand(amax_shape, generator=g) * 3 + 0.1
    amax.view(-1)[0] = 0.0  # one zero-amax channel
    ref = R.tensor_quant(x, amax, 8, False, False)
    out = ops().quantize_op(x.to(gpu), amax.to(gpu), 8, 0, False, False)
    assert same_bits(out, ref), mismatch(out, ref)


def test_int_with_axis_api(gpu):
    x = rand_with_edges((48, 96), torch.bfloat16, seed=2)
    amax = torch.rand(96) + 0.5
    ref = R.tensor_quant(x, amax.view(1, 96), 8, False, True)
    out = ops().fake_tensor_quant_with_axis(x.to(gpu), amax.to(gpu), 1, 8, False, True)
    assert same_bits(out, ref), mismatch(out, ref)


def test_int_inplace(gpu):
    x = rand_with_edges((1000,), torch.float16, seed=4)
    amax = torch.tensor(1.5)
    ref = R.tensor_quant(x, amax, 8, False, True)
    xd = x.to(gpu)
    ops().fake_tensor_quant_(xd, amax.to(gpu), 8, False, True)
    assert same_bits(xd, ref), mismatch(xd, ref)


def test_int_bf16_amax_dtype(gpu):
    # amax kept in the input dtype (MaxCalibrator output) is read directly by the kernel
    x = rand_with_edges((128, 64), torch.bfloat16, seed=9)
    amax = x.abs().amax(dim=1, keepdim=True)
    ref = R.tensor_quant(x, amax, 8, False, False)
    out = ops().quantize_op(x.to(gpu), amax.to(gpu), 8, 0, False, False)
    assert same_bits(out, ref), mismatch(out, ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("fmt", ["int8", "int4", "fp8"])
@pytest.mark.parametrize("shape", [(16, 2048), (6, 1024), (96, 4096)])
def test_long_rows_own_dtype_amax(gpu, dtype, fmt, shape):
    """A bf16 / f16 model's per-channel weight amax is kept in the weight's dtype (MaxCalibrator):
    the wave-uniform row kernel reads it in that dtype (mtq_dispatch_counts shows ew_rowwave)."""
    from modelopt_amd import _ext

    x = rand_with_edges(shape, dtype, seed=21)
    amax = x.abs().amax(dim=1, keepdim=True)
    amax.view(-1)[1] = 0.0
    before = _ext.dispatch_counts()["ew_rowwave"]
    if fmt == "fp8":
        ref = R.fp8_eager(x, amax)
        out = ops().quantize_op(x.to(gpu), amax.to(gpu), 8, 4, False, False)
    else:
        bits = 8 if fmt == "int8" else 4
        ref = R.tensor_quant(x, amax, bits, False, False)
        out = ops().quantize_op(x.to(gpu), amax.to(gpu), bits, 0, False, False)
    assert same_bits(out, ref), mismatch(out, ref)
    assert _ext.dispatch_counts()["ew_rowwave"] == before + 1


# --------------------------------------------------------------------------------------------
# FP8
# --------------------------------------------------------------------------------------------


@pytest.mark.parametrize("dtype", DTYPES)
def test_fp8_per_tensor(gpu, dtype):
    x = rand_with_edges((257, 129), dtype, seed=1, scale=3.0)
    amax = x.float().abs().amax() * 0.5  # clip half of the range
    ref = R.fp8_eager(x, amax)
    out = ops().fake_e4m3fy(x.to(gpu), amax.to(gpu))
    assert same_bits(out, ref), mismatch(out, ref)


def test_fp8_special_values(gpu):
    vals = [448.0, 449.0, 463.99, 464.0, 465.0, 480.0, 1e9, float("inf"), -float("inf"),
            float("nan"), 0.0, -0.0, 2.0**-9, 2.0**-10, 1.5 * 2.0**-10, 2.0**-7 * 1.0625]
    x = torch.tensor(vals, dtype=torch.float32)
    for amax in [448.0, 0.0, 1e-30, 3.0]:
        a = torch.tensor(amax)
        ref = R.fp8_eager(x, a)
        out = ops().fake_e4m3fy(x.to(gpu), a.to(gpu))
        assert same_bits(out, ref), (amax, mismatch(out, ref))


def test_fp8_exhaustive_bf16(gpu):
    # every finite bf16 value through the per-tensor FP8 path at several scales
    bits = torch.arange(0, 1 << 16, dtype=torch.int32).to(torch.int16)
    x = bits.view(torch.bfloat16)
    for amax in [448.0, 1.0, 3.1415, 1e-3, 6e4]:
        a = torch.tensor(amax)
        ref = R.fp8_eager(x, a)
        out = ops().fake_e4m3fy(x.to(gpu), a.to(gpu))
        assert same_bits(out, ref), (amax, mismatch(out, ref))


def test_e4m3_cast(gpu):
    bits = torch.arange(0, 1 << 16, dtype=torch.int32).to(torch.int16)
    x = bits.view(torch.bfloat16)
    ref = R.fp8_eager(x, None)
    out = ops().e4m3_cast(x.to(gpu))
    assert same_bits(out, ref), mismatch(out, ref)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize(
    "shape,amax_shape",
    [((64, 256), (64, 1)), ((64, 256), (1, 256)), ((8192, 128), (8192, 1)), ((16, 2048), (16, 1))],
)
def test_fp8_axis_and_block(gpu, dtype, shape, amax_shape):
    x = rand_with_edges(shape, dtype, seed=21, scale=2.0)
    g = torch.Generator().manual_seed(8)
    amax = torch.rand(amax_shape, generator=g) * 4 + 0.01
    amax.view(-1)[1] = 0.0
    ref = R.fp8_eager(x, amax)
    out = ops().quantize_op(x.to(gpu), amax.to(gpu), 8, 4, False, False)
    assert same_bits(out, ref), mismatch(out, ref)


# --------------------------------------------------------------------------------------------
# MX dynamic block
# --------------------------------------------------------------------------------------------

MX_FORMATS = ["E2M1", "E3M2", "E2M3", "E4M3", "E5M2", "INT8", "E1M2", "E0M3", "E3M0"]


@pytest.mark.parametrize("fmt", MX_FORMATS)
@pytest.mark.parametrize("bs", [8, 16, 32])
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("cols", [128, 100])
def test_mx_vs_oracle(gpu, fmt, bs, dtype, cols):
    g = torch.Generator().manual_seed(bs + cols)
    x = (torch.randn(33, cols, generator=g) * torch.logspace(-3, 3, cols)).to(dtype)
    x[0, :bs] = 0.0
    x[1, 0] = 6.0 * 2**3  # amax exactly at emax * 2^k
    ref = R.fused_amax_convert(x, bs, fmt)
    out = ops().fused_amax_convert(x.to(gpu), bs, R.FORMAT_CODES[fmt], R.FORMAT_CODES["E8M0"], None)
    assert torch.equal(out.cpu().float(), ref.float()) or same_bits(out, ref), mismatch(out, ref)


def _all_16bit_patterns(dtype, order):
    """Every bf16 / f16 bit pattern as one [2048, 32] tensor: "sorted" by magnitude (blocks of
    like exponents: every E8M0 / E4M3 scale regime incl. subnormal and huge blocks, the NaN / inf
    patterns together at the end), "shuffled" (NaN, inf, -0 spread over many blocks) or
    "finite" (shuffled, no NaN / inf)."""
    bits = torch.arange(65536, dtype=torch.int32).to(torch.int16)
    x = bits.view(dtype)
    if order == "sorted":
        x = x[torch.argsort(x.float().abs().nan_to_num(float("inf")), stable=True)]
    elif order == "shuffled":
        x = x[torch.randperm(65536, generator=torch.Generator().manual_seed(3))]
    else:
        x = x[torch.isfinite(x.float())]
        x = x[torch.randperm(x.numel(), generator=torch.Generator().manual_seed(4))]
        x = x[: x.numel() // 32 * 32]
    return x.reshape(-1, 32).contiguous()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("order", ["sorted", "shuffled", "finite"])
@pytest.mark.parametrize("bs", [8, 16, 32])
def test_mxfp4_native_convert_all_patterns(gpu, dtype, order, bs):
    """The native-FP4-convert MXFP4 path (mx_e2m1_native_kernel) vs the KAT-pinned oracle on
    every 16-bit input pattern: -0, NaN of both signs, inf, subnormals, every scale exponent."""
    x = _all_16bit_patterns(dtype, order)
    ref = R.fused_amax_convert(x, bs, "E2M1")
    out = ops().fused_amax_convert(x.to(gpu), bs, R.FORMAT_CODES["E2M1"], R.FORMAT_CODES["E8M0"], None)
    assert same_bits(out, ref), mismatch(out, ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("order", ["sorted", "shuffled", "finite"])
def test_nvfp4_native_convert_all_patterns(gpu, dtype, order):
    """The native-FP4-convert NVFP4 path (nvfp4_native_kernel) vs the oracle on every 16-bit
    input pattern, at several global amax values (block scales from 1e-12 to saturated)."""
    x = _all_16bit_patterns(dtype, order)
    fin = x.float().abs()
    fin = fin[torch.isfinite(fin)]
    for ga in (fin.amax(), torch.tensor(1.0), torch.tensor(0.0), fin.amax() * 1e-6):
        ref = R.nvfp4_fake_quant_block(x, ga)
        out = ops().nvfp4_fake_quant_block(x.to(gpu), ga.to(gpu).float(), 16)
        assert same_bits(out, ref), (float(ga), mismatch(out, ref))


def test_mx_blocksize_error(gpu):
    x = torch.randn(4, 64, device=gpu)
    with pytest.raises(ValueError):
        ops().fused_amax_convert(x, 64, R.FORMAT_CODES["E2M1"], R.FORMAT_CODES["E8M0"], None)


# --------------------------------------------------------------------------------------------
# amax reductions
# --------------------------------------------------------------------------------------------


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize(
    "shape,axis",
    [
        ((1 << 20) + 7, None),
        ((512, 4096), None),
        ((512, 4096), 0),  # keep rows: reduce each row (weight per-channel)
        ((512, 4096), -1),  # keep columns
        ((4, 96, 16), 1),  # keep the middle
        ((4, 96, 16), (0, 1)),  # keep leading run
        ((3000, 128), 0),  # block view rows of 128
        ((64, 3), -1),  # generic small
        ((7, 5, 3), (1,)),
    ],
)
def test_reduce_amax(gpu, dtype, shape, axis):
    from modelopt_amd.torch.quantization.utils.core_utils import reduce_amax

    shape = (shape,) if isinstance(shape, int) else shape
    g = torch.Generator().manual_seed(len(shape))
    x = (torch.randn(shape, generator=g) * 3).to(dtype)
    raxis = R.convert_quantization_axis_to_reduce_axis(x, axis)
    ref = R.reduce_amax(x, axis=raxis)
    out = reduce_amax(x.to(gpu), axis=raxis)
    assert out.shape == ref.shape and out.dtype == ref.dtype
    assert same_bits(out, ref), mismatch(out, ref)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize(
    "shape,axis",
    [
        ((5000, 4104), -1),  # columns: a partial last 64-vector chunk
        ((3000, 96), -1),  # columns: fewer than 64 vectors across (many row lanes)
        ((70000, 64), -1),  # columns: long and narrow (slab count capped by rows)
        ((1001, 128), 0),  # short rows: R not a multiple of the rows per block
        ((37, 14344), 0),  # long rows: several chunks per row, partial last chunk
        ((6, 5, 40), (0, 2)),  # short rows with P > 1 (atomic fold onto r % K)
    ],
)
def test_reduce_amax_launch_shapes(gpu, dtype, shape, axis):
    """Edge shapes of the wide-column, unrolled-row and short-row amax launches."""
    from modelopt_amd.torch.quantization.utils.core_utils import reduce_amax

    g = torch.Generator().manual_seed(sum(shape))
    x = (torch.randn(shape, generator=g) * 3).to(dtype)
    x.view(-1)[:: 997] *= 50  # scattered outliers
    raxis = R.convert_quantization_axis_to_reduce_axis(x, axis)
    ref = R.reduce_amax(x, axis=raxis)
    out = reduce_amax(x.to(gpu), axis=raxis)
    assert same_bits(out, ref), mismatch(out, ref)
    # accumulation into an existing running max (the calibrator's fold), twice the same input
    from modelopt_amd.torch.quantization.utils.core_utils import reduce_amax_accumulate

    acc = torch.zeros(ref.numel(), dtype=torch.float32, device=gpu)
    xg = x.to(gpu)
    reduce_amax_accumulate(xg, acc, raxis)
    reduce_amax_accumulate(xg * 0.5, acc, raxis)
    assert torch.equal(acc.cpu(), ref.float().reshape(-1))


def test_reduce_amax_nan_inf(gpu):
    from modelopt_amd.torch.quantization.utils.core_utils import reduce_amax

    x = torch.randn(1000, 64)
    x[10, 3] = float("nan")
    x[20, 5] = -float("inf")
    for axis in [None, [1], [0]]:
        ref = R.reduce_amax(x, axis=axis)
        out = reduce_amax(x.to(gpu), axis=axis)
        assert same_bits(out, ref), (axis, mismatch(out, ref))


# --------------------------------------------------------------------------------------------
# histogram
# --------------------------------------------------------------------------------------------


@pytest.mark.parametrize("bins", [2048, 3001, 20000])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_histogram_matches_histc(gpu, bins, dtype):
    g = torch.Generator().manual_seed(bins)
    x = (torch.randn(1 << 18, generator=g) * 2).to(dtype)
    xa = x.float().abs()
    hmax = xa.max()
    ref = torch.histc(xa, bins=bins, min=0, max=float(hmax))
    counts = torch.zeros(bins, dtype=torch.int32, device=gpu)
    ops().histogram_abs_accumulate(x.to(gpu), hmax.to(gpu).float(), counts, bins, False)
    assert torch.equal(counts.cpu().float(), ref), (counts.cpu().float() - ref).abs().max()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("bins", [64, 2048, 4096, 8192, 9000])
@pytest.mark.parametrize("skip_zeros", [False, True])
def test_histogram_16bit_table_path(gpu, dtype, bins, skip_zeros):
    """The per-block bin table of the 16-bit path: zeros, values at / above the range end,
    NaN / inf, subnormals, every bin-count regime (REP 8 / 4 / 2 / 1)."""
    g = torch.Generator().manual_seed(bins + skip_zeros)
    x = (torch.randn(1 << 17, generator=g) * 2).to(dtype)
    x[:500] = 0
    x[500:510] = float("nan")
    x[510:520] = float("inf")
    x[520:600] = torch.finfo(dtype).tiny / 4  # subnormals
    hmax = x[600:].float().abs().max() * 0.9  # some finite values lie above the range
    x[600:610] = hmax.to(dtype)
    xa = x.float().abs()
    keep = ~torch.isnan(xa) & (xa <= hmax)
    if skip_zeros:
        keep &= xa != 0
    ref = torch.histc(xa[keep], bins=bins, min=0, max=float(hmax))
    counts = torch.zeros(bins, dtype=torch.int32, device=gpu)
    ops().histogram_abs_accumulate(x.to(gpu), hmax.to(gpu).float(), counts, bins, skip_zeros)
    assert torch.equal(counts.cpu().float(), ref), (counts.cpu().float() - ref).abs().max()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_histogram_pattern_path_many_blocks(gpu, dtype):
    """The 16-bit pattern histogram over many blocks, a ragged last block chunk and heavy-tailed
    data (hot bins), vs torch.histc."""
    g = torch.Generator().manual_seed(7)
    n = 8 * ((1 << 21) + 3)
    x = torch.randn(n, generator=g)
    x[:: 997] *= 16
    x = x.to(dtype)
    xa = x.float().abs()
    hmax = xa.max()
    ref = torch.histc(xa, bins=2048, min=0, max=float(hmax))
    counts = torch.zeros(2048, dtype=torch.int32, device=gpu)
    ops().histogram_abs_accumulate(x.to(gpu), hmax.to(gpu).float(), counts, 2048, False)
    assert torch.equal(counts.cpu().float(), ref), (counts.cpu().float() - ref).abs().max()


def test_histogram_degenerate_range(gpu):
    x = torch.zeros(1000)
    ref = torch.histc(x, bins=64, min=0, max=0)
    counts = torch.zeros(64, dtype=torch.int32, device=gpu)
    ops().histogram_abs_accumulate(x.to(gpu), torch.zeros((), device=gpu), counts, 64, False)
    assert torch.equal(counts.cpu().float(), ref)


# --------------------------------------------------------------------------------------------
# fused dynamic INT block quant (AWQ weight side)
# --------------------------------------------------------------------------------------------


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("with_pqs", [False, True])
def test_block_quant_dynamic(gpu, dtype, with_pqs):
    g = torch.Generator().manual_seed(1)
    w = (torch.randn(96, 512, generator=g) * 0.02).to(dtype)
    pqs = (torch.rand(512, generator=g) + 0.5).to(dtype) if with_pqs else None
    ref = R.int_block_qdq_dynamic(w, 128, 4, pqs)
    out = ops().block_quant_dynamic(w.to(gpu), None if pqs is None else pqs.to(gpu), 128, 4, False, False)
    assert same_bits(out, ref), mismatch(out, ref)


def test_reduce_amax_unaligned_and_chunk_edges(gpu):
    """Per-tensor amax: 16 B-misaligned views (scalar path) and sizes around the chunk size."""
    from modelopt_amd.torch.quantization.utils.core_utils import reduce_amax

    g = torch.Generator().manual_seed(7)
    for n in [1, 7, 8, 2047, 2048 * 8, 2048 * 8 + 1, 3 * 2048 * 8 - 9, 1 << 21]:
        base = torch.randn(n + 1, generator=g).to(torch.bfloat16)
        for x in (base[:n], base[1:]):
            ref = R.reduce_amax(x, axis=None)
            out = reduce_amax(x.to(gpu) if x.storage_offset() == 0 else base.to(gpu)[1:], axis=None)
            assert same_bits(out, ref), (n, x.storage_offset(), mismatch(out, ref))


# --------------------------------------------------------------------------------------------
# AWQ-lite search helpers: column scale and the per-alpha MSE
# --------------------------------------------------------------------------------------------


@pytest.mark.parametrize("dtype", DTYPES)
def test_mul_cols(gpu, dtype):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(37, 4, 256, generator=g).to(dtype)
    s = (torch.rand(256, generator=g) + 0.25).to(dtype)
    out = ops().mul_cols(x.to(gpu), s.to(gpu))
    assert same_bits(out, x * s), mismatch(out, x * s)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n", [5, 4096, 12345, 1 << 22])
def test_mse_accumulate(gpu, dtype, n):
    """loss[i] += (a - b).float().pow(2).mean(): the difference is rounded to dtype exactly as
    the reference does; only the summation order differs (tolerance 1e-5 relative)."""
    g = torch.Generator().manual_seed(n)
    a = torch.randn(n, generator=g).to(dtype)
    b = (a.float() + 0.01 * torch.randn(n, generator=g)).to(dtype)
    ref = (a - b).float().pow(2).double().mean()
    loss = torch.zeros(3, device=gpu)
    ops().mse_accumulate(a.to(gpu), b.to(gpu), loss, 1)
    got = loss.cpu().double()
    assert got[0] == 0 and got[2] == 0
    torch.testing.assert_close(got[1], ref, rtol=1e-5, atol=0)
    # deterministic: a second accumulation from the same start gives the same bits
    loss2 = torch.zeros(3, device=gpu)
    ops().mse_accumulate(a.to(gpu), b.to(gpu), loss2, 1)
    assert torch.equal(loss, loss2)


# --------------------------------------------------------------------------------------------
# NVFP4 (E2M1 elements, E4M3 block scales, fp32 global amax)
# --------------------------------------------------------------------------------------------


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(64, 128), (33, 48), (7, 40), (5, 3, 64), (1, 5)])
def test_nvfp4_kernel_vs_oracle(gpu, dtype, shape):
    g = torch.Generator().manual_seed(sum(shape))
    x = (torch.randn(shape, generator=g) * torch.logspace(-3, 2, shape[-1])).to(dtype)
    x.view(-1)[:3] = torch.tensor([0.0, -0.0, 1e-30]).to(dtype)
    for ga in (x.float().abs().amax(), torch.tensor(0.0), x.float().abs().amax() * 100):
        ref = R.nvfp4_fake_quant_block(x, ga)
        out = ops().nvfp4_fake_quant_block(x.to(gpu), ga.to(gpu), 16)
        assert same_bits(out, ref), (float(ga), mismatch(out, ref))


def test_nvfp4_kernel_vs_reference_golden(gpu):
    """The reference's own fp4_fake_quant_block outputs (tests/golden/nvfp4.*)."""
    import json as _json
    from pathlib import Path

    from safetensors.torch import load_file

    gold = Path(__file__).resolve().parent / "golden"
    t = load_file(str(gold / "nvfp4.safetensors"))
    for name, m in _json.loads((gold / "nvfp4.json").read_text()).items():
        if "blocks" not in m:
            continue
        x, amax, y, ok = t[f"{name}.x"], t[f"{name}.amax"], t[f"{name}.y"], t[f"{name}.block_ok"].bool()
        out = ops().nvfp4_fake_quant_block(x.to(gpu), amax.to(gpu), 16).cpu()
        okc = ok.repeat_interleave(16, dim=1)[:, : x.shape[-1]]
        assert torch.equal(out[okc], y[okc]), name
        # on the excluded blocks the HIP kernel equals the oracle (hardware RNE cast)
        assert same_bits(out, R.nvfp4_fake_quant_block(x, amax)), name


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("cols", [64, 40])
@pytest.mark.parametrize("per_channel", [False, True])
def test_mx_two_level_scale_vs_oracle(gpu, dtype, cols, per_channel):
    """fused_amax_convert with E4M3 block scales and a global amax (compute_scale_with_global)."""
    g = torch.Generator().manual_seed(cols)
    x = (torch.randn(24, cols, generator=g) * torch.logspace(-2, 2, cols)).to(dtype)
    ga = x.float().abs().amax(dim=1) if per_channel else x.float().abs().amax().reshape(1)
    if per_channel and cols % 16:
        pytest.skip("per-channel with padded blocks indexes past the rows in the reference (UB)")
    ref = R.fused_amax_convert(x, 16, "E2M1", "E4M3", ga)
    out = ops().fused_amax_convert(x.to(gpu), 16, R.FORMAT_CODES["E2M1"], R.FORMAT_CODES["E4M3"], ga.to(gpu))
    assert same_bits(out, ref), mismatch(out, ref)


def test_nvfp4_quantizer_dispatch(gpu):
    """NVFP4 dynamic TensorQuantizer -> fp4_fake_quant_block semantics (block 16, global amax =
    the calibrated / dynamic per-tensor amax); DISABLE_TRITON_KERNEL -> fused_amax_convert."""
    from modelopt_amd.torch.quantization import tensor_quant as tqm
    from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig
    from modelopt_amd.torch.quantization.nn import TensorQuantizer

    cfg = QuantizerAttributeConfig(num_bits=(2, 1), block_sizes={-1: 16, "type": "dynamic", "scale_bits": (4, 3)})
    q = TensorQuantizer(cfg).to(gpu)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(32, 64, generator=g).to(torch.bfloat16)
    out = q(x.to(gpu))
    ga = x.float().abs().amax()
    assert same_bits(out, R.nvfp4_fake_quant_block(x, ga.to(torch.bfloat16).float()))
    try:
        tqm.DISABLE_TRITON_KERNEL = True
        out2 = q(x.to(gpu))
    finally:
        tqm.DISABLE_TRITON_KERNEL = False
    ref2 = R.fused_amax_convert(x, 16, "E2M1", "E4M3", ga.to(torch.bfloat16).float().reshape(1))
    assert same_bits(out2, ref2), mismatch(out2, ref2)


@pytest.mark.parametrize("dtype", DTYPES)
def test_fp4_block_scale_quant_vs_oracle(gpu, dtype):
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(40, 32, generator=g) * 3).to(dtype)
    scale = torch.rand(40 * 2, generator=g) * 0.5
    scale[:4] = torch.tensor([0.0, float("nan"), float("inf"), 1e-30])
    ref = R.nvfp4_scalar_quant(x.reshape(80, 16), scale.view(80, 1)).reshape(x.shape).to(dtype)
    out = ops().fp4_block_scale_quant(x.to(gpu), scale.to(gpu))
    assert same_bits(out, ref), mismatch(out, ref)
    # ragged: block not a multiple of the vector -> scalar kernel
    x2 = torch.randn(9, 20, generator=g).to(dtype)
    s2 = torch.rand(9, generator=g)
    ref2 = R.nvfp4_scalar_quant(x2, s2.view(9, 1)).to(dtype)
    assert same_bits(ops().fp4_block_scale_quant(x2.to(gpu), s2.to(gpu)), ref2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_nvfp4_static_quantizer(gpu, dtype):
    """NVFP4 static weight quantizer: max-calibrated per-block amax, promoted with global amax =
    max(per-block amax) (core_utils.py:1077-1150), then the two-level static fake quant."""
    import torch.nn as nn

    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.nn.modules.tensor_quantizer import StaticBlockScaleQuantizer

    g = torch.Generator().manual_seed(12)
    lin = nn.Linear(64, 48, bias=False).to(dtype)
    with torch.no_grad():
        lin.weight.copy_((torch.randn(48, 64, generator=g) * torch.logspace(-2, 0, 64)).to(dtype))
    w = lin.weight.detach().clone()
    lin.to(gpu)
    cfg = {
        "quant_cfg": [
            {"quantizer_name": "*", "enable": False},
            {"quantizer_name": "*weight_quantizer",
             "cfg": {"num_bits": (2, 1), "block_sizes": {-1: 16, "type": "static", "scale_bits": (4, 3)}}},
        ],
        "algorithm": "max",
    }
    mtq.quantize(lin, cfg, lambda m: m(torch.randn(4, 64, device=gpu, dtype=dtype)))
    q = lin.weight_quantizer
    assert isinstance(q, StaticBlockScaleQuantizer)
    amax = w.float().reshape(-1, 16).abs().amax(dim=1, keepdim=True)
    assert torch.equal(q.amax.cpu(), amax) and torch.equal(q.global_amax.cpu(), amax.amax())
    out = q(lin.weight)
    ref = R.static_blockwise_fp4_fake_quant(w.reshape(-1, 16), amax, amax.amax()).reshape(w.shape)
    assert same_bits(out, ref), mismatch(out, ref)


# --------------------------------------------------------------------------------------------
# checkpoint export packing
# --------------------------------------------------------------------------------------------


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(96, 256), (10, 24), (7, 13)])
def test_export_fp8_vs_oracle(gpu, dtype, shape):
    g = torch.Generator().manual_seed(shape[0])
    w = (torch.randn(shape, generator=g) * 0.05).to(dtype)
    w.view(-1)[:4] = torch.tensor([0.0, -0.0, 10.0, -10.0]).to(dtype)  # 10 / s overflows -> NaN
    s = w.float().abs().amax() / 448
    ref = R.export_fp8(w, s)
    out = ops().export_fp8(w.to(gpu), s.to(gpu), False, True).view(torch.uint8).cpu()
    assert torch.equal(out, ref)
    srow = w.float().abs().amax(dim=1) / 448
    ref2 = R.export_fp8(w, srow[:, None])
    out2 = ops().export_fp8(w.to(gpu), srow.to(gpu), True, False).view(torch.uint8).cpu()
    assert torch.equal(out2, ref2)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape,block", [((64, 256), 128), ((6, 40), 8), ((4, 12), 4)])
def test_export_int4_vs_oracle(gpu, dtype, shape, block):
    g = torch.Generator().manual_seed(block)
    w = (torch.randn(shape, generator=g) * 0.05).to(dtype)
    s = w.float().reshape(shape[0], -1, block).abs().amax(-1) / 7
    ref = R.export_int4(w, s)
    out = ops().export_int4(w.to(gpu), s.to(gpu)).cpu()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(64, 256), (5, 48), (3, 2, 32)])
def test_export_nvfp4_vs_oracle(gpu, dtype, shape):
    g = torch.Generator().manual_seed(sum(shape))
    w = (torch.randn(shape, generator=g) * 0.05).to(dtype)
    s2 = w.float().abs().amax() / 2688
    bs = (w.float().reshape(*shape[:-1], -1, 16).abs().amax(-1) / (6 * s2)).clamp(2**-9, 448)
    bs = bs.to(torch.float8_e4m3fn).float()
    ref = R.export_nvfp4(w, bs, s2)
    out = ops().export_nvfp4(w.to(gpu), bs.to(gpu), s2.to(gpu)).cpu()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("dtype", DTYPES)
# (37, 4096) / (33, 8224): several 1024-vector workgroups and a partial last one (the packer's
# LDS-gathered scale line falls back to byte stores there; 8481 blocks is not a multiple of 4)
@pytest.mark.parametrize("shape", [(64, 256), (3, 96), (37, 4096), (33, 8224)])
def test_export_mxfp4_vs_oracle(gpu, dtype, shape):
    g = torch.Generator().manual_seed(shape[1])
    w = (torch.randn(shape, generator=g) * torch.logspace(-3, 1, shape[1])).to(dtype)
    w[0, :32] = 0  # an all-zero block: exponent clamps at -127, zeros carry the sign bit
    ref_q, ref_s = R.export_mxfp4(w, 32)
    q, s = ops().export_mxfp4(w.to(gpu), 32)
    assert torch.equal(q.cpu(), ref_q) and torch.equal(s.cpu().reshape(-1), ref_s.reshape(-1))
