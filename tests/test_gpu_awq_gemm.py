"""AWQ-lite alpha-search GEMM on MFMA (csrc/mtq_awq_gemm.hip, C ABI mtq_awq_search_gemm).

The kernel computes, for every alpha g of one linear,
    loss[g] += mean((T(T(x * sinv[g]) @ wq[g]^T + bias) - yref)^2)      (model_calib.py:1489-1560)
without storing the GEMM output.  Checks:

* exact data (small integers: every fp32 product sum is exact, so the bf16 output is the correctly
  rounded value on any summation order): the loss equals an fp64 host evaluation of the same
  expression bit for bit -- this pins the fragment layouts, the LDS swizzle, the XCD remap, the
  alpha grouping, bias, tails in M and N, and the rounding of x * sinv and of the difference;
* random bf16 data at Llama shapes: loss within rtol 2e-3 of the unfused path (x * sinv, then
  hipBLASLt F.linear, then the loss in fp32) -- the fp32 accumulation orders differ, which moves a
  few outputs by one bf16 ulp; the bound is stated here and is far below the 10-100 % spread
  between the alphas' losses that the search ranks;
* the weight side ``block_quant_dynamic_multi`` equals G single-alpha launches bit for bit.
Both search kernels run every check: ``kernel=1`` the r03 ping-pong kernel (8 waves), ``kernel=2``
the r06 one-wave-per-SIMD kernel whose K loop is generated inline asm (scripts/gen_awq_w4.py; K >=
128, K % 128 == 0); ``kernel=0`` (what the product calls) is the second where its limits allow.
"""

import pytest
import torch
import torch.nn.functional as F

from modelopt_amd import _ext

pytestmark = pytest.mark.gpu


def ops():
    return _ext.ops()


def _host_loss(x, sinv, wq, bias, yref):
    """fp64 evaluation of the fused expression with the reference's roundings (dtype of x)."""
    dt = x.dtype
    out = []
    for g in range(wq.shape[0]):
        xs = (x.float() * sinv[g].float()).to(dt)
        y = xs.double() @ wq[g].double().t()
        if bias is not None:
            y = y + bias.double()
        y = y.float().to(dt)  # exact-data case: y.double() is exact, float() exact, one rounding
        d = (y.float() - yref.float()).to(dt).double()
        out.append((d * d).sum() / d.numel())
    return torch.tensor(out, dtype=torch.float64).float()


@pytest.mark.parametrize("kernel", [1, 2])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(256, 256, 64), (300, 320, 192), (512, 768, 256), (37, 1024, 128),
                                   (1000, 520, 640)])
@pytest.mark.parametrize("with_bias", [False, True])
def test_exact_integer_data(gpu, dtype, shape, with_bias, kernel):
    M, N, K = shape
    if kernel == 2 and K % 128:
        pytest.skip("the W4 kernel needs K % 128 == 0 (test_kernel_choice covers the rejection)")
    G = 3
    g = torch.Generator().manual_seed(M + N + K)
    # sparse small integers: every product sum, output, difference and square sum (per lane,
    # per tile) is an integer below 2^24, so fp32 arithmetic is exact in any order
    x = (torch.randint(-1, 2, (M, K), generator=g) * (torch.rand(M, K, generator=g) < 0.125)).to(dtype)
    sinv = torch.tensor([1.0, 0.5, 2.0]).view(G, 1).expand(G, K).contiguous().to(dtype)
    wq = torch.randint(-1, 2, (G, N, K), generator=g).to(dtype)
    # asymmetric in every index so a transposed or permuted layout cannot pass
    wq[1, :, 0] = torch.arange(N).remainder(3).to(dtype)
    x[:, 1] = torch.arange(M).remainder(3).to(dtype)
    bias = torch.randint(-2, 3, (N,), generator=g).to(dtype) if with_bias else None
    yref = torch.randint(-4, 5, (M, N), generator=g).to(dtype)
    loss = torch.zeros(G, device=gpu)
    ops().awq_search_gemm(x.to(gpu), sinv.to(gpu), wq.to(gpu), None if bias is None else bias.to(gpu),
                          yref.to(gpu), loss, kernel)
    want = _host_loss(x, sinv, wq, bias, yref)
    assert torch.equal(loss.cpu(), want), (loss.cpu(), want)
    # accumulates (loss[g] += ...) and is deterministic
    ops().awq_search_gemm(x.to(gpu), sinv.to(gpu), wq.to(gpu), None if bias is None else bias.to(gpu),
                          yref.to(gpu), loss, kernel)
    assert torch.equal(loss.cpu(), want + want)


@pytest.mark.parametrize("kernel", [1, 2])
@pytest.mark.parametrize("nk", [(1024, 4096), (4096, 4096), (14336, 4096), (4096, 14336)])
def test_llama_shapes_vs_unfused(gpu, nk, kernel):
    N, K = nk
    M, G = 512, 4
    dt = torch.bfloat16
    gen = torch.Generator(device=gpu).manual_seed(N + K)
    x = torch.randn(M, K, device=gpu, generator=gen).to(dt)
    w = (torch.randn(N, K, device=gpu, generator=gen) * 0.02).to(dt)
    bias = (torch.randn(N, device=gpu, generator=gen) * 0.1).to(dt)
    s = torch.rand(G, K, device=gpu, generator=gen) * 3 + 0.25
    pqs_w, sinv = s.to(dt), (1 / s).to(dt)
    wq = ops().block_quant_dynamic_multi(w, pqs_w, 128, 4, False, False)
    for gi in (0, G - 1):
        assert torch.equal(wq[gi], ops().block_quant_dynamic(w, pqs_w[gi], 128, 4, False, False))
    yref = F.linear(x, w, bias)
    loss = torch.zeros(G, device=gpu)
    ops().awq_search_gemm(x, sinv, wq, bias, yref, loss, kernel)
    want = torch.stack([(F.linear(x * sinv[gi], wq[gi], bias) - yref).float().pow(2).mean() for gi in range(G)])
    torch.testing.assert_close(loss, want, rtol=2e-3, atol=0)
    again = torch.zeros(G, device=gpu)
    ops().awq_search_gemm(x, sinv, wq, bias, yref, again, kernel)
    assert torch.equal(loss, again)  # deterministic
    # the two kernels hold the same fp32 accumulators (same MFMA k order); only the per-tile
    # square-sum order differs
    other = torch.zeros(G, device=gpu)
    ops().awq_search_gemm(x, sinv, wq, bias, yref, other, 3 - kernel)
    torch.testing.assert_close(loss, other, rtol=1e-5, atol=0)


def test_kernel_choice(gpu):
    """kernel=0 (the product call) runs the W4 kernel where K % 128 == 0 and the ping-pong kernel
    otherwise; asking for W4 at K = 64 is an error, not a silent fallback."""
    from modelopt_amd import _ext as ext

    dt = torch.bfloat16
    for K, kernel, want in ((64, 0, "awq_search_pp"), (192, 0, "awq_search_pp"), (4096, 0, "awq_search_w4"),
                            (128, 2, "awq_search_w4"), (4096, 1, "awq_search_pp")):
        x = torch.randn(256, K, device=gpu).to(dt)
        wq = torch.randn(2, 256, K, device=gpu).to(dt)
        sinv = torch.ones(2, K, device=gpu, dtype=dt)
        before = ext.dispatch_counts()
        ops().awq_search_gemm(x, sinv, wq, None, torch.zeros(256, 256, device=gpu, dtype=dt),
                              torch.zeros(2, device=gpu), kernel)
        torch.cuda.synchronize()
        after = ext.dispatch_counts()
        grown = {k for k in after if after[k] > before.get(k, 0)}
        assert want in grown and ({"awq_search_pp", "awq_search_w4"} - {want}).isdisjoint(grown), (K, grown)
    with pytest.raises(RuntimeError):
        ops().awq_search_gemm(torch.zeros(256, 64, device=gpu, dtype=dt), torch.ones(2, 64, device=gpu, dtype=dt),
                              torch.zeros(2, 256, 64, device=gpu, dtype=dt), None,
                              torch.zeros(256, 256, device=gpu, dtype=dt), torch.zeros(2, device=gpu), 2)


def test_rejects_unsupported(gpu):
    x = torch.zeros(8, 96, device=gpu, dtype=torch.bfloat16)  # K % 64 != 0
    wq = torch.zeros(1, 16, 96, device=gpu, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops().awq_search_gemm(x, torch.ones(1, 96, device=gpu, dtype=torch.bfloat16), wq, None,
                              torch.zeros(8, 16, device=gpu, dtype=torch.bfloat16), torch.zeros(1, device=gpu))


class _Mlp(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.up = torch.nn.Linear(512, 1024)
        self.mid = torch.nn.Linear(1024, 2048, bias=False)
        self.down = torch.nn.Linear(2048, 512)

    def forward(self, x):
        return self.down(torch.relu(self.mid(torch.relu(self.up(x)))))


def _awq_run(gpu, mode):
    import copy

    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization import model_calib

    torch.manual_seed(5)
    m = _Mlp().to(gpu).to(torch.bfloat16)
    g = torch.Generator(device=gpu).manual_seed(9)
    data = [torch.randn(2, 96, 512, device=gpu, generator=g).to(torch.bfloat16) for _ in range(3)]
    cfg = copy.deepcopy(mtq.INT4_AWQ_CFG)
    cfg["algorithm"] = {"method": "awq_lite", "alpha_step": 0.1, "debug": True}
    old = model_calib._AWQ_FUSED
    model_calib._AWQ_FUSED = mode
    try:
        mtq.quantize(m, cfg, lambda mm: [mm(d) for d in data])
    finally:
        model_calib._AWQ_FUSED = old
    return m


@pytest.mark.parametrize("mode", ["always", "auto", "library"])
def test_awq_lite_fused_search_matches_per_alpha_path(gpu, mode):
    """awq_lite end to end with the fused MFMA search ("always"; "auto" sends the 2048-wide
    linear and narrower ones to it and the rest to batched hipBLASLt + the multi-alpha loss pass)
    vs the per-alpha hipBLASLt path ("never"): per-alpha losses within rtol 2e-3 (GEMM summation
    order), the same best alpha, and then the same scales, weights and amax bit for bit."""
    fused, ref = _awq_run(gpu, mode), _awq_run(gpu, "never")
    for name in ("up", "mid", "down"):
        hf, hr = getattr(fused, name).awq_lite, getattr(ref, name).awq_lite
        torch.testing.assert_close(hf.loss, hr.loss, rtol=2e-3, atol=0)
        assert hf.best_alpha == hr.best_alpha, name
        assert torch.equal(hf.best_scale, hr.best_scale)
        assert torch.equal(getattr(fused, name).weight, getattr(ref, name).weight)
        assert torch.equal(getattr(fused, name).weight_quantizer.amax, getattr(ref, name).weight_quantizer.amax)


@pytest.mark.parametrize("G", [1, 11, 16])
def test_prescale_and_mse_multi(gpu, G):
    gen = torch.Generator(device=gpu).manual_seed(G)
    x = torch.randn(300, 512, device=gpu, generator=gen).to(torch.bfloat16)
    s = (torch.rand(G, 512, device=gpu, generator=gen) + 0.5).to(torch.bfloat16)
    xs = _ext.ops().awq_prescale(x, s)
    for g in range(G):
        assert torch.equal(xs[g], x * s[g])  # the reference's bf16 multiply, bit for bit
    ref = torch.randn(300, 256, device=gpu, generator=gen).to(torch.bfloat16)
    out = torch.randn(G, 300, 256, device=gpu, generator=gen).to(torch.bfloat16)
    loss = torch.zeros(G, device=gpu)
    _ext.ops().awq_mse_multi(out, ref, loss)
    want = torch.stack([(out[g] - ref).float().pow(2).mean() for g in range(G)])
    torch.testing.assert_close(loss, want, rtol=1e-5, atol=0)
    again = torch.zeros(G, device=gpu)
    _ext.ops().awq_mse_multi(out, ref, again)
    assert torch.equal(loss, again)



def test_w4_bitwise_repeatable_under_load(gpu):
    """The W4 kernel's waits and barriers are counted by hand (scripts/gen_awq_w4.py); a read placed
    before its data landed shows as run-to-run differences under contention.  20 back-to-back
    launches at a Llama shape (11 alphas, full-chip grid, the tail tiles' reference DMAs) must give
    bit-identical losses, equal to the ping-pong kernel's within the square-sum order."""
    M, N, K, G = 2048, 4096, 4096, 11
    dt = torch.bfloat16
    gen = torch.Generator(device=gpu).manual_seed(77)
    x = torch.randn(M, K, device=gpu, generator=gen).to(dt)
    w = (torch.randn(N, K, device=gpu, generator=gen) * 0.02).to(dt)
    s = torch.rand(G, K, device=gpu, generator=gen) * 3 + 0.25
    wq = ops().block_quant_dynamic_multi(w, s.to(dt), 128, 4, False, False)
    si = (1 / s).to(dt)
    yref = F.linear(x, w)
    runs = []
    for _ in range(20):
        loss = torch.zeros(G, device=gpu)
        ops().awq_search_gemm(x, si, wq, None, yref, loss, 2)
        runs.append(loss)
    torch.cuda.synchronize()
    for r in runs[1:]:
        assert torch.equal(r, runs[0])
    pp = torch.zeros(G, device=gpu)
    ops().awq_search_gemm(x, si, wq, None, yref, pp, 1)
    torch.testing.assert_close(runs[0], pp, rtol=1e-5, atol=0)
