"""The fused QuantLinear simulated GEMM for short inputs (csrc/mtq_qlinear.hip, MFMA).

Two properties pin it:
* bit-exact weight fake quant: with one-hot input rows (x[m] = e_k) every output element is a
  single product 1 * qdq(W)[n, k], exact in the fp32 accumulator and in the output dtype, so the
  in-register qdq is compared bit for bit with the oracle's qdq of W (oracle/ref_ops.py, pinned to
  the reference) at those columns;
* the GEMM: random inputs against an fp64 product of the same operands (x and the oracle's
  qdq(W)), within the fp32-accumulation + one-output-rounding bound, and against the unfused
  module path (F.linear on hipBLASLt).
The module-level tests check that QuantLinear takes the fused path for short inputs with the
reference's configs and gives the unfused path's result.
"""

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu


def ops():
    from modelopt_amd import _ext

    return _ext.ops()


def oracle_wq(w, amax, block, kind, num_bits=8, unsigned=False, narrow=False):
    """qdq(W) on the CPU oracle with the kernel's amax layout."""
    n, k = w.shape
    wc = w.cpu()
    a = amax.cpu()
    if a.numel() == 1:
        am, view = a.reshape(()), wc
    else:
        view = wc.reshape(-1, block)
        am = a.reshape(-1, 1)
    if kind == 1:
        out = R.fp8_eager(view, am)
    else:
        out = R.tensor_quant(view, am, num_bits, unsigned, narrow)
    return out.reshape(n, k)


CASES = [
    # (kind, num_bits, unsigned, narrow, amax layout)
    (0, 8, False, False, "channel"),
    (0, 8, False, True, "tensor"),
    (0, 4, False, False, "block128"),
    (0, 4, True, False, "block64"),
    (1, 8, False, False, "tensor"),
    (1, 8, False, False, "channel"),
    (1, 8, False, False, "block128"),
]


def make_amax(w, layout):
    n, k = w.shape
    if layout == "tensor":
        return w.float().abs().amax().reshape(()) * 0.9, k
    if layout == "channel":
        return w.float().abs().amax(dim=1, keepdim=True) * 0.9, k
    b = int(layout[5:])
    return w.float().reshape(-1, b).abs().amax(dim=1, keepdim=True) * 0.9, b


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES)
def test_weight_qdq_bit_exact_through_one_hot_rows(gpu, dtype, case):
    kind, nb, uns, narrow, layout = case
    n, k = 48, 256
    g = torch.Generator().manual_seed(3)
    w = (torch.randn(n, k, generator=g) * 0.05).to(dtype)
    if uns:
        w = w.abs()
    amax, block = make_amax(w, layout)
    cols = torch.tensor([0, 1, 31, 32, 63, 64, 127, 128, 129, 200, 255] + list(range(2, 7)))  # 16 rows
    x = torch.zeros(len(cols), k, dtype=dtype)
    x[torch.arange(len(cols)), cols] = 1.0
    y = ops().qlinear_small_m(x.to(gpu), w.to(gpu), None, amax.to(gpu), block, kind, nb, uns, narrow)
    want = oracle_wq(w, amax, block, kind, nb, uns, narrow)[:, cols].t().contiguous()
    # value equality: a -0 weight comes out as +0 after the sum with the other waves' zeros
    assert torch.equal(y.cpu().float(), want.float())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m", [1, 3, 9, 16])
@pytest.mark.parametrize(
    "nk,case",
    [(nk, c) for nk in [(16, 32), (48, 96), (256, 1024), (128, 4096)]
     for c in [CASES[0], CASES[2], CASES[4], CASES[6]]
     if not (c[4].startswith("block") and nk[1] % int(c[4][5:]))],  # blocks must tile K
)
@pytest.mark.parametrize("with_bias", [False, True])
def test_gemm_against_fp64(gpu, dtype, m, nk, case, with_bias):
    kind, nb, uns, narrow, layout = case
    n, k = nk
    g = torch.Generator().manual_seed(m * 7 + n + k)
    w = (torch.randn(n, k, generator=g) * 0.05).to(dtype)
    x = torch.randn(m, k, generator=g).to(dtype)
    b = (torch.randn(n, generator=g) * 0.1).to(dtype) if with_bias else None
    amax, block = make_amax(w, layout)
    y = ops().qlinear_small_m(x.to(gpu), w.to(gpu), None if b is None else b.to(gpu), amax.to(gpu),
                              block, kind, nb, uns, narrow).cpu()
    wq = oracle_wq(w, amax, block, kind, nb, uns, narrow)
    exact = x.double() @ wq.double().t() + (0 if b is None else b.double())
    # fp32 accumulation of k exact products + bias, then one rounding to the output dtype
    mag = x.double().abs() @ wq.double().abs().t() + (0 if b is None else b.double().abs())
    ulp = 2.0 ** -7 if dtype == torch.bfloat16 else 2.0 ** -10
    bound = exact.abs() * ulp + mag * (k + 2) * 2.0 ** -24 + 1e-30
    err = (y.double() - exact).abs()
    assert bool((err <= bound).all()), float((err / bound).max())


def test_rejects_unsupported_shapes(gpu):
    x = torch.randn(2, 40, device=gpu, dtype=torch.bfloat16)
    w = torch.randn(16, 40, device=gpu, dtype=torch.bfloat16)
    a = torch.ones((), device=gpu)
    with pytest.raises(RuntimeError, match="invalid argument"):
        ops().qlinear_small_m(x, w, None, a, 40, 0, 8, False, False)  # K % 32 != 0
    x = torch.randn(17, 64, device=gpu, dtype=torch.bfloat16)
    w = torch.randn(16, 64, device=gpu, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="invalid argument"):
        ops().qlinear_small_m(x, w, None, a, 64, 0, 8, False, False)  # M > 16


@pytest.mark.parametrize("cfg_name", ["INT8_DEFAULT_CFG", "FP8_DEFAULT_CFG", "INT4_AWQ_CFG", "W4A8_AWQ_BETA_CFG"])
@pytest.mark.parametrize("tokens", [1, 7, 16])
def test_quant_linear_short_inputs_take_fused_path(gpu, cfg_name, tokens, monkeypatch):
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.nn.modules import quant_linear as ql

    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(256, 512), nn.ReLU(), nn.Linear(512, 128, bias=False)).to(gpu, torch.bfloat16)
    calib = [torch.randn(4, 33, 256, device=gpu, dtype=torch.bfloat16) for _ in range(2)]
    mtq.quantize(model, getattr(mtq, cfg_name), lambda m: [m(c) for c in calib])
    x = torch.randn(tokens, 256, device=gpu, dtype=torch.bfloat16)
    calls = []
    real = ql._fused_forward

    def spy(mod, inp):
        out = real(mod, inp)
        calls.append(out is not None)
        return out

    monkeypatch.setattr(ql, "_fused_forward", spy)
    with torch.no_grad():
        fused = model(x)
        ql._FUSED[0] = False
        try:
            unfused = model(x)
        finally:
            ql._FUSED[0] = True
    # W4A8 stacks two weight quantizers (SequentialQuantizer): the reference path runs
    want_fused = cfg_name != "W4A8_AWQ_BETA_CFG"
    assert calls[:2] == [want_fused, want_fused], calls
    tol = 2 ** -6
    assert torch.allclose(fused.float(), unfused.float(), rtol=tol, atol=tol * unfused.float().abs().max().item())


def test_quant_linear_long_inputs_and_grad_use_reference_path(gpu):
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.nn.modules import quant_linear as ql

    model = nn.Linear(128, 64).to(gpu, torch.bfloat16)
    mtq.quantize(model, mtq.INT8_DEFAULT_CFG, lambda m: m(torch.randn(8, 128, device=gpu, dtype=torch.bfloat16)))
    assert ql._fused_forward(model, torch.randn(17, 128, device=gpu, dtype=torch.bfloat16)) is None
    x = torch.randn(4, 128, device=gpu, dtype=torch.bfloat16, requires_grad=True)
    assert ql._fused_forward(model, x) is None
    model(x).sum().backward()
    assert x.grad is not None


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m", [1, 5, 16])
@pytest.mark.parametrize("case", [CASES[1], CASES[2], CASES[4], CASES[5]])
def test_group_launch_against_fp64(gpu, dtype, m, case):
    """q/k/v-shaped linears (different N, same K and input rows) in one grouped launch: each
    output within the single kernel's fp32-accumulation bound of its own fp64 product, bias on one
    of them, per-linear amax (and for INT-n per-linear num_bits flags)."""
    kind, nb, uns, narrow, layout = case
    k = 1024
    g = torch.Generator().manual_seed(m + 11 * kind)
    ns = [256, 64, 64]
    ws = [(torch.randn(n, k, generator=g) * 0.05).to(dtype) for n in ns]
    xs = [torch.randn(m, k, generator=g).to(dtype) for _ in ns]
    bs = [None, (torch.randn(64, generator=g) * 0.1).to(dtype), None]
    am = [make_amax(w, layout) for w in ws]
    ys = ops().qlinear_small_m_group([x.to(gpu) for x in xs], [w.to(gpu) for w in ws],
                                     [None if b is None else b.to(gpu) for b in bs], [a.to(gpu) for a, _ in am],
                                     [blk for _, blk in am], kind, [nb] * 3, [int(uns)] * 3, [int(narrow)] * 3)
    ulp = 2.0 ** -7 if dtype == torch.bfloat16 else 2.0 ** -10
    for x, w, b, (a, blk), y in zip(xs, ws, bs, am, ys):
        wq = oracle_wq(w, a, blk, kind, nb, uns, narrow)
        exact = x.double() @ wq.double().t() + (0 if b is None else b.double())
        mag = x.double().abs() @ wq.double().abs().t() + (0 if b is None else b.double().abs())
        bound = exact.abs() * ulp + mag * (k + 2) * 2.0 ** -24 + 1e-30
        err = (y.cpu().double() - exact).abs()
        assert y.shape == (m, w.shape[0])
        assert bool((err <= bound).all()), float((err / bound).max())


def test_group_launch_one_hot_bit_exact_and_mixed_fallback(gpu):
    """One-hot rows through the grouped launch give the oracle's qdq(W) bit for bit; a group whose
    linears differ in kind runs them one after another with the same results."""
    k = 256
    g = torch.Generator().manual_seed(5)
    ws = [(torch.randn(n, k, generator=g) * 0.05).to(torch.bfloat16) for n in (48, 32)]
    cols = torch.tensor([0, 1, 31, 32, 63, 64, 127, 128, 129, 200, 255, 2, 3, 4, 5, 6])
    x = torch.zeros(16, k, dtype=torch.bfloat16)
    x[torch.arange(16), cols] = 1.0
    for kinds in ((1, 1), (0, 1)):
        ams = [make_amax(w, "tensor") for w in ws]
        if kinds[0] != kinds[1]:
            ys = [ops().qlinear_small_m_group([x.to(gpu)], [w.to(gpu)], [None], [a.to(gpu)], [blk], kd, [8], [0], [0])[0]
                  for w, (a, blk), kd in zip(ws, ams, kinds)]
        else:
            ys = ops().qlinear_small_m_group([x.to(gpu)] * 2, [w.to(gpu) for w in ws], [None, None],
                                             [a.to(gpu) for a, _ in ams], [blk for _, blk in ams], kinds[0],
                                             [8, 8], [0, 0], [0, 0])
        for w, (a, blk), kd, y in zip(ws, ams, kinds, ys):
            want = oracle_wq(w, a, blk, kd)[:, cols].t().contiguous()
            assert torch.equal(y.cpu().float(), want.float())


@pytest.mark.parametrize("family", ["llama", "qwen2"])  # qwen2: q/k/v projections with biases
@pytest.mark.parametrize("cfg_name", ["FP8_DEFAULT_CFG", "INT4_AWQ_CFG"])
def test_attention_qkv_projections_run_as_one_launch(gpu, cfg_name, family, monkeypatch):
    """A decode step of a quantized HF Llama / Qwen2 runs q/k/v_proj as one grouped launch (one
    take that launches, two that hand out cached outputs) and its logits match the ungrouped fused
    path."""
    import transformers

    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.nn.modules import quant_linear as ql

    cfg_cls, model_cls = ((transformers.LlamaConfig, transformers.LlamaForCausalLM) if family == "llama"
                          else (transformers.Qwen2Config, transformers.Qwen2ForCausalLM))
    cfg = cfg_cls(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                  num_key_value_heads=2, vocab_size=128, max_position_embeddings=64)
    torch.manual_seed(0)
    model = model_cls(cfg).to(gpu, torch.bfloat16).eval()
    if family == "qwen2":
        assert model.model.layers[0].self_attn.q_proj.bias is not None
    ids = torch.randint(0, 128, (2, 4, 16), device=gpu)
    mtq.quantize(model, getattr(mtq, cfg_name), lambda m: [m(b) for b in ids])
    counts = {"grouped": 0, "cached": 0}
    real_take = ql.ProjectionGroup.take

    def spy(self, mod, inp):
        had_key = self.key is not None
        y = real_take(self, mod, inp)
        if y is not None:
            counts["cached" if had_key else "grouped"] += 1
        return y

    monkeypatch.setattr(ql.ProjectionGroup, "take", spy)
    x = torch.randint(0, 128, (1, 1), device=gpu)
    with torch.no_grad():
        grouped = model(x).logits
        monkeypatch.setattr(ql.ProjectionGroup, "take", lambda self, mod, inp: None)
        single = model(x).logits
    assert counts == {"grouped": 2, "cached": 4}, counts  # per layer: one launch, two cached outputs
    tol = 2 ** -6
    assert torch.allclose(grouped.float(), single.float(), rtol=tol, atol=tol * single.float().abs().max().item())


def _qkv_group(gpu, cfg_name):
    import modelopt_amd.torch.quantization as mtq

    torch.manual_seed(3)
    mods = [nn.Linear(256, n).to(gpu, torch.bfloat16) for n in (256, 128, 128)]
    calib = torch.randn(4, 8, 256, device=gpu, dtype=torch.bfloat16)
    for m in mods:
        mtq.quantize(m, getattr(mtq, cfg_name), lambda mm: mm(calib))
    return mods


@pytest.mark.parametrize("cfg_name", ["FP8_DEFAULT_CFG", "INT8_DEFAULT_CFG"])
def test_projection_group_k_v_with_other_input(gpu, cfg_name):
    """q launches the group on its input; k/v then called with a DIFFERENT tensor (a
    cross-attention key_value_states) drop the cached outputs and compute on their own input --
    outputs equal the ungrouped path, and no input quantizer collected a foreign tensor."""
    from modelopt_amd.torch.quantization.nn.modules import quant_linear as ql

    mods = _qkv_group(gpu, cfg_name)
    xq = torch.randn(1, 256, device=gpu, dtype=torch.bfloat16)
    xkv = torch.randn(1, 256, device=gpu, dtype=torch.bfloat16) * 3
    with torch.no_grad():
        want = [mods[0](xq), mods[1](xkv), mods[2](xkv)]
        grp = ql.ProjectionGroup(mods)
        for m in mods:
            m.__dict__["_projection_group"] = grp
        try:
            got = [mods[0](xq), mods[1](xkv), mods[2](xkv)]
        finally:
            for m in mods:
                m.__dict__.pop("_projection_group", None)
    assert grp.key is not None  # q did launch the group
    for a, b in zip(got, want):
        tol = 2 ** -6
        assert torch.allclose(a.float(), b.float(), rtol=tol, atol=tol * b.float().abs().max().item())


def test_projection_group_not_used_while_input_quantizers_calibrate(gpu):
    """A calibrating input quantizer has a side effect (it collects): the group must not apply it to
    q's input on behalf of k/v -- each collects its own input."""
    from modelopt_amd.torch.quantization.nn.modules import quant_linear as ql

    mods = _qkv_group(gpu, "FP8_DEFAULT_CFG")
    for m in mods:
        m.input_quantizer.enable_calib()
    assert not any(ql._input_quantizer_pure(m) for m in mods)
    grp = ql.ProjectionGroup(mods)
    x = torch.randn(1, 256, device=gpu, dtype=torch.bfloat16)
    assert grp.take(mods[0], x) is None and grp.key is None
