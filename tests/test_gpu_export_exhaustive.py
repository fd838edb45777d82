"""Checkpoint-export packers over every 16-bit input pattern, bit for bit against the oracle.

The packers take native gfx950 fast paths (v_cvt_scalef32_pk_fp4_f32 for the E2M1 codes, packed
v_cvt_pk_fp8_f32 for e4m3) and fall back to the exact emulated conversion only on the lanes where
the converter and the reference can disagree (csrc/mtq_kernels.hip, "Native fast paths").  These
tests sweep the inputs where that matters:
  * MXFP4 (qtensor/mxfp4_tensor.py:38-81, ties toward zero): every bf16 / f16 pattern at block
    exponents from the fallback region (e < -100, all-zero blocks) to e = 126 (inf / NaN patterns
    excluded: their blocks' scale byte is NaN cast to uint8, unspecified in the reference);
  * NVFP4 (qtensor/nvfp4_tensor.py:230-342, ties to the even code): fp32 quotients within a few
    ulps of every E2M1 grid point and midpoint (divisor 1, so q = x exactly), and every bf16 pattern
    divided by non-power-of-two block scales (full-mantissa quotients);
  * FP8 (export/quant_utils.py:855-913): every bf16 / f16 pattern over per-tensor and per-row scales,
    the (448, 464] rounding band and the NaN / overflow bytes.
The emulated path is covered here by the lanes that fall back (NaN / overflow quotients, zero divisors, tiny block exponents).
"""

import pytest
import torch

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu


def _ops():
    from modelopt_amd import _ext

    return _ext.ops()


def all_patterns(dtype):
    """Every 16-bit pattern of `dtype` as a 1-D tensor of that dtype."""
    return torch.arange(-32768, 32768, dtype=torch.int32).to(torch.int16).view(dtype)


def mxfp4_blocks(dtype, anchor):
    """Blocks of 32: element 0 = anchor (sets the block amax unless a pattern exceeds it),
    elements 1..31 walk every pattern of dtype."""
    p = all_patterns(dtype)
    p = torch.where(torch.isfinite(p.float()), p, torch.zeros((), dtype=dtype))  # inf/NaN: below
    pad = (-p.numel()) % 31
    p = torch.cat([p, torch.zeros(pad, dtype=dtype)]).view(-1, 31)
    a = torch.full((p.shape[0], 1), anchor, dtype=torch.float32).to(dtype)
    return torch.cat([a, p], dim=1).contiguous()  # [blocks, 32]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_export_mxfp4_every_pattern(gpu, dtype):
    fmax = torch.finfo(dtype).max
    ks = [-133, -127, -110, -101, -100, -99, -60, -20, -3, -1, 0, 1, 2, 7, 30, 90, 125, 126]
    anchors = []
    for k in ks:
        for m in (6.0, 5.0, 4.0, 7.5, 3.0):
            v = m * 2.0**k
            t = torch.tensor(v, dtype=torch.float32).to(dtype)
            if torch.isfinite(t) and float(t) != 0.0 and float(t) <= fmax:
                anchors.append(float(t))
    anchors = sorted(set(anchors))
    x = torch.cat([mxfp4_blocks(dtype, a) for a in anchors])
    x = torch.cat([x, torch.zeros(2, 32, dtype=dtype)])  # all-zero blocks (e = -127)
    ref_q, ref_s = R.export_mxfp4(x, 32)
    q, s = _ops().export_mxfp4(x.to(gpu), 32)
    q, s = q.cpu(), s.cpu().reshape(-1)
    bad = (q != ref_q).nonzero()
    assert bad.numel() == 0, (len(bad), bad[:4].tolist(), x.view(-1, 32)[bad[:4, 0]].float()[:, :4])
    assert torch.equal(s, ref_s.reshape(-1))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_export_mxfp4_mixed_vectors(gpu, dtype):
    """Random blocks where a few lanes hold zeros or hit exact midpoints, beside lanes that do not:
    the per-lane fallback must not disturb neighbours."""
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4096, 32, generator=g) * torch.logspace(-4, 3, 4096)[:, None]
    e = torch.ceil(torch.log2(x.abs().amax(1, keepdim=True) / 6))
    mids = torch.tensor([0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5.0, 0.5, 1.0, 6.0])
    idx = torch.randint(0, 32, (4096, 3), generator=g)
    sel = mids[torch.randint(0, len(mids), (4096, 3), generator=g)] * torch.exp2(e)
    sel = sel * torch.where(torch.rand(4096, 3, generator=g) < 0.5, -1.0, 1.0)
    x.scatter_(1, idx, sel)
    x[::5, 3] = 0.0
    x[::7, 9] = -0.0
    x = x.to(dtype)
    ref_q, ref_s = R.export_mxfp4(x, 32)
    q, s = _ops().export_mxfp4(x.to(gpu), 32)
    assert torch.equal(q.cpu(), ref_q) and torch.equal(s.cpu().reshape(-1), ref_s.reshape(-1))


def _near(v, k=6):
    """fp32 values within k ulps of v (both signs)."""
    b = torch.tensor([v], dtype=torch.float32).view(torch.int32)
    r = (b + torch.arange(-k, k + 1, dtype=torch.int32)).view(torch.float32)
    return torch.cat([r, -r])


def test_export_nvfp4_fp32_near_every_bound(gpu):
    pts = [0.0, 0.25, 0.5, 0.75, 1.0, 1.25, 1.5, 1.75, 2.0, 2.5, 3.0, 3.5, 4.0, 5.0, 6.0, 6.5, 1e30]
    vals = torch.cat([_near(v) for v in pts[1:]] + [torch.tensor([0.0, -0.0, 1e-45, -1e-45])])
    vals = torch.cat([vals, torch.tensor([float("inf"), -float("inf"), float("nan"), 3e38, -3e38])])
    n = vals.numel()
    vals = torch.cat([vals, torch.zeros((-n) % 32)]).view(-1, 32)
    bs = torch.ones(vals.shape[0], 2)
    s2 = torch.tensor(1.0)
    ref = R.export_nvfp4(vals, bs, s2)
    out = _ops().export_nvfp4(vals.to(gpu), bs.to(gpu), s2.to(gpu)).cpu()
    assert torch.equal(out, ref), (out != ref).nonzero()[:8].tolist()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("s2v", [1.0, 0.3, 7.77e-3])
def test_export_nvfp4_every_pattern(gpu, dtype, s2v):
    p = all_patterns(torch.bfloat16 if dtype == torch.float32 else dtype).to(dtype)
    x = p.view(-1, 64)  # 1024 rows x 4 blocks of 16
    g = torch.Generator().manual_seed(int(s2v * 1000))
    bs = (torch.rand(x.shape[0], 4, generator=g) * 400 + 0.01).to(torch.float8_e4m3fn).float()
    bs[::9] = 0.0  # zero block scale: the lane falls back (q = x / 0)
    s2 = torch.tensor(s2v)
    ref = R.export_nvfp4(x, bs, s2)
    out = _ops().export_nvfp4(x.to(gpu), bs.to(gpu), s2.to(gpu)).cpu()
    assert torch.equal(out, ref), (out != ref).nonzero()[:8].tolist()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_export_fp8_every_pattern(gpu, dtype):
    x = all_patterns(dtype).view(-1, 256)
    # A NaN weight is a NaN byte (0x7F | sign); torch's CPU cast of a bf16 NaN to float8_e4m3fn
    # sets the sign bit for positive NaNs too (f16 and fp32 keep it), an x86 artefact the device
    # does not copy, so NaN inputs are checked for the NaN byte only.
    nan = torch.isnan(x.float())
    for sv in (1.0, 0.0123, 3.7, 1.0 / 448):
        s = torch.tensor(sv)
        ref = R.export_fp8(x, s)
        out = _ops().export_fp8(x.to(gpu), s.to(gpu), False, True).view(torch.uint8).cpu()
        assert bool(((out & 0x7F) == 0x7F)[nan].all())
        ref = torch.where(nan, out, ref)
        assert torch.equal(out, ref), (sv, (out != ref).nonzero()[:8].tolist())
    srow = torch.logspace(-3, 2, x.shape[0])
    ref2 = R.export_fp8(x, srow[:, None])
    out2 = _ops().export_fp8(x.to(gpu), srow.to(gpu), True, False).view(torch.uint8).cpu()
    assert torch.equal(out2, ref2), (out2 != ref2).nonzero()[:8].tolist()


def test_export_fp8_rounding_band(gpu):
    """Quotients in and around (448, 464]: 448 below the tie at 464, NaN above; per-row fp32."""
    v = torch.cat([_near(448.0, 4), _near(456.0, 4), _near(464.0, 4), _near(480.0, 2),
                   torch.tensor([float("nan"), float("inf"), -float("inf"), 0.0, -0.0, 1e-9])])
    n = v.numel()
    x = torch.cat([v, torch.zeros((-n) % 8)]).view(-1, 8)
    srow = torch.ones(x.shape[0])
    ref = R.export_fp8(x, srow[:, None])
    out = _ops().export_fp8(x.to(gpu), srow.to(gpu), True, False).view(torch.uint8).cpu()
    assert torch.equal(out, ref), (out != ref).nonzero()[:8].tolist()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_export_int4_every_pattern(gpu, dtype):
    """pack_int4_in_uint8 (export/quant_utils.py:792-833) over every pattern, +-inf / NaN included,
    with zero and tiny per-block scales (those lanes divide with the IEEE operator)."""
    x = all_patterns(dtype).view(512, 128)
    g = torch.Generator().manual_seed(3)
    s = torch.rand(512, 128 // 32, generator=g) * 0.5 + 1e-3
    s[::11] = 0.0
    s[5::13] = 1e-39  # reciprocal overflows to inf
    ref = R.export_int4(x, s)
    out = _ops().export_int4(x.to(gpu), s.to(gpu)).cpu()
    assert torch.equal(out, ref), (out != ref).nonzero()[:8].tolist()
