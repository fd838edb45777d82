"""The calibration bookkeeping kernels (mtq_amax_fill / _fold / _check, csrc/mtq_kernels.hip) that
replace torch.zeros / torch.maximum / isnan-isinf-any on the running-max buffers: same values as
the torch expressions they replace, and MaxCalibrator / _validate_quantizer_attrs behave as before
(reference calib/max.py:53-86 asserts, tensor_quantizer.py:757-773 validate_attr)."""
import math

import pytest
import torch

from modelopt_amd import _ext

pytestmark = pytest.mark.gpu


def test_fill_fold_match_torch(gpu):
    ops = _ext.ops()
    for n in (1, 7, 4096, 100003):
        t = torch.full((n,), 3.0, device=gpu)
        ops.amax_fill_(t, 0.0)
        assert torch.equal(t, torch.zeros(n, device=gpu))
        g = torch.Generator(device=gpu).manual_seed(n)
        a = torch.rand(n, device=gpu, generator=g) * 10
        b = torch.rand(n, device=gpu, generator=g) * 10
        if n > 4:
            a[1], b[2], a[3], b[3] = math.nan, math.nan, math.inf, math.nan
        want = torch.maximum(a, b)
        ops.amax_fold_(a, b)
        nan = torch.isnan(want)
        assert torch.equal(torch.isnan(a), nan) and torch.equal(a[~nan], want[~nan])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_check_flags(gpu, dtype):
    ops = _ext.ops()
    # above 2^20 elements the grid-stride form (zeroed flags, 16-byte vectors, a ragged tail);
    # the [1:] view is not 16-byte aligned: the one-workgroup form
    for n in (1, 1000, 70001, (1 << 20) + 1, 3_000_007, -3_000_001):
        x = (torch.rand(abs(n) + (n < 0), device=gpu) + 0.5).to(dtype)
        if n < 0:
            x, n = x[1:], -n
        assert ops.amax_check(x).tolist() == [0, 0, 0]
        for pos, val, flag in ((n - 1, math.nan, 0), (n // 2, -math.inf, 1), (0, -0.25, 2)):
            y = x.clone()
            y[pos] = val
            want = [0, 0, 0]
            want[flag] = 1
            if flag == 1:
                want[2] = 1  # -inf is also negative
            assert ops.amax_check(y).tolist() == want, (n, pos, val)
    assert ops.amax_check(torch.empty(0, device=gpu, dtype=dtype)).tolist() == [0, 0, 0]


def test_max_calibrator_nan_inf_asserts(gpu):
    from modelopt_amd.torch.quantization.calib.max import MaxCalibrator

    for bad, msg in ((math.nan, "nan"), (math.inf, "inf")):
        c = MaxCalibrator()
        x = torch.ones(64, device=gpu, dtype=torch.bfloat16)
        x[5] = bad
        c.collect(x)
        with pytest.raises(AssertionError, match=msg):
            c.compute_amax()
    c = MaxCalibrator()
    c.collect(torch.full((64,), -2.0, device=gpu))
    assert float(c.compute_amax()) == 2.0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cols", [64, 4096, 37])
def test_mask_unrouted_rows_matches_where(gpu, dtype, cols):
    """_QuantFusedExperts' masking of rows routed to no local expert: the library pass equals
    torch.where(any(0 <= idx < E), hs, 0) bit for bit (NaN rows kept when routed, +0 otherwise)."""
    ops = _ext.ops()
    g = torch.Generator(device=gpu).manual_seed(cols)
    T, E, k = 300, 8, 2
    hs = torch.randn(T, cols, device=gpu, generator=g).to(dtype)
    hs[3, 1] = math.nan
    hs[4, 0] = -0.0
    idx = torch.randint(0, E, (T, k), device=gpu, generator=g)
    idx[::5, 0] = -1  # sentinel in one slot: still routed through the other
    idx[::7] = E  # both slots outside the local experts: masked
    idx[4] = -1
    routed = ((idx >= 0) & (idx < E)).any(dim=-1, keepdim=True)
    want = torch.where(routed, hs, hs.new_zeros(()))
    got = ops.mask_unrouted_rows(hs, idx, E)
    iv = torch.int32 if dtype == torch.float32 else torch.int16
    assert torch.equal(got.view(iv), want.view(iv))
