"""MXFP8 (E4M3 elements, E8M0 block scales) fake quant on the native gfx950 scaled converts
(mx_e4m3_native_kernel) against the emulated path (mx_vec_kernel, the restatement of
tensor_quant_mx.cu:36-55, 104-137 that the oracle pins; tests/test_gpu_golden.py).

The emulated kernel computes in fp32 from the exactly widened 16-bit input and rounds once to the
output dtype, so the 16-bit native result must equal ``fused_amax_convert(x.float()).to(dtype)`` bit
for bit.  Exhaustive: every 16-bit pattern (NaN, inf, -0 and subnormals included) inside blocks
whose amax pins every block exponent the dtype can reach, plus blocks of random magnitudes."""

import pytest
import torch

from modelopt_amd import _ext

pytestmark = pytest.mark.gpu


def _all_patterns_at_every_scale(dtype, dev):
    pats = torch.arange(-32768, 32768, dtype=torch.int32).to(torch.int16).view(dtype)
    vals = pats.float().abs()
    finite_max = torch.finfo(dtype).max
    blocks = []
    for e in range(-160, 130):
        a = 448.0 * 2.0**e
        anchor = torch.tensor([a], dtype=torch.float32).to(dtype)
        if not torch.isfinite(anchor).all() or float(anchor) == 0 or float(anchor) > finite_max:
            continue
        # the patterns at or below the anchor (NaN / inf patterns go with the first block set only)
        keep = (vals <= float(anchor)) if blocks else torch.ones_like(vals, dtype=torch.bool)
        p = pats[keep]
        p = p[torch.randperm(p.numel(), generator=torch.Generator().manual_seed(e + 200))]
        pad = (-p.numel()) % 31
        p = torch.cat([p, torch.zeros(pad, dtype=dtype)]).view(-1, 31)
        blocks.append(torch.cat([anchor.expand(p.shape[0], 1), p], dim=1))
    return torch.cat(blocks).reshape(-1).to(dev)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_mxfp8_native_equals_emulated_exhaustive(gpu, dtype):
    ops = _ext.ops()
    x = _all_patterns_at_every_scale(dtype, gpu)
    before = _ext.dispatch_counts()
    got = ops.fused_amax_convert(x, 32, 0, 9, None)
    after = _ext.dispatch_counts()
    assert after["mx_e4m3_native"] == before["mx_e4m3_native"] + 1
    want = ops.fused_amax_convert(x.float(), 32, 0, 9, None).to(dtype)
    # NaN blocks run the same emulated code in both kernels; only the NaN payload of the fp32 ->
    # 16-bit cast of `want` (torch) differs from the kernel's store, so NaN matches NaN
    gi, wi = got.view(torch.int16), want.view(torch.int16)
    bad = ((gi != wi) & ~(torch.isnan(got) & torch.isnan(want))).nonzero().view(-1)
    assert bad.numel() == 0, (bad.numel(), x[bad[:8]].tolist(), got[bad[:8]].tolist(), want[bad[:8]].tolist())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(4096, 4096), (7, 32), (3, 96)])
def test_mxfp8_native_random_blocks(gpu, dtype, shape):
    ops = _ext.ops()
    g = torch.Generator(device=gpu).manual_seed(17)
    x = torch.randn(shape, device=gpu, generator=g)
    # block magnitudes spread over many octaves (f16: inside its range)
    span = 20 if dtype == torch.float16 else 120
    mag = torch.exp2(torch.randint(-span // 2, span // 2, (x.numel() // 32, 1), device=gpu, generator=g).float())
    x = (x.view(-1, 32) * mag).view(shape).to(dtype)
    x.view(-1)[5] = -0.0
    got = ops.fused_amax_convert(x, 32, 0, 9, None)
    want = ops.fused_amax_convert(x.float(), 32, 0, 9, None).to(dtype)
    same = (got.view(torch.int16) == want.view(torch.int16)) | (torch.isnan(got) & torch.isnan(want))
    assert bool(same.all())
