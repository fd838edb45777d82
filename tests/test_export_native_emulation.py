"""Host proof of the MXFP4 export packer's native fast path (csrc/mtq_kernels.hip,
export_mxfp4_vec_one): for a 16-bit weight x and block exponent e, the gfx950 converter's
round-to-nearest-even-code of (x - 1 fp32 ulp) / 2^e, with quotients that are zero in fp32 patched
to code 8, equals the reference's strict-bound count (qtensor/mxfp4_tensor.py:46-53: ties toward
zero, sign(0) = 0 -> sign bit set).  The converter's RNE is modelled exactly in float64 (the
probe in profiles/r02/fp4_convert_probe.txt and tests/test_gpu_export_exhaustive.py pin the
hardware to that model); this test sweeps every finite bf16 / f16 pattern over the native
exponent range in numpy, in a few seconds.
"""

import numpy as np
import pytest

GRID = np.array([0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0])
BOUNDS = np.array([0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5.0])


def rne_code(a):
    """E2M1 magnitude code of a >= 0 (float64): nearest, ties to the even code, saturating."""
    k = np.clip(np.searchsorted(GRID, a, side="right") - 1, 0, 6)
    mid = (GRID[k] + GRID[k + 1]) / 2
    c = np.where(a < mid, k, np.where(a > mid, k + 1, k + (k % 2)))
    return np.where(a >= 6.0, 7, c)


def patterns(dtype):
    p = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    if dtype == "bf16":
        f = (p.astype(np.uint32) << 16).view(np.float32)
    else:
        f = p.view(np.float16).astype(np.float32)
    return f[np.isfinite(f)]


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_mxfp4_native_rounding_model(dtype):
    x = patterns(dtype)
    for e in list(range(-100, -90)) + list(range(-30, 31)) + list(range(118, 128)):
        # reference: q = x / 2^e in fp32, code = 8 * ((2 - sign(q)) // 2) + #(bounds < |q|)
        with np.errstate(over="ignore"):  # |x| far above the block amax: both saturate to 7
            q = (x / np.float32(2.0**e)).astype(np.float32)
        ref = np.where(q > 0, 0, 8) + (np.abs(q)[:, None] > BOUNDS).sum(1)
        # kernel: converter RNE on (x - 1 ulp) / 2^e, sign from the operand, zero quotients -> 8
        xd = (x.view(np.uint32) - np.uint32(1)).view(np.float32).astype(np.float64)
        hw = rne_code(np.abs(xd) / 2.0**e) + np.where(np.signbit(xd), 8, 0)
        zthr = 2.0 ** (e - 150) if e >= 1 else 0.0
        hw = np.where(np.abs(x.astype(np.float64)) <= zthr, 8, hw)
        bad = np.nonzero(hw != ref)[0]
        assert bad.size == 0, (dtype, e, x[bad[:4]], hw[bad[:4]], ref[bad[:4]])
