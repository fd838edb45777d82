"""Calibration searches on the GPU: MSE calibrators (calib/mse.py) and AWQ-clip
(model_calib.py:1725-1940) vs the CPU oracle and the reference's own outputs (tests/golden/mse.*,
tests/golden/awq_clip.*, made by running the reference; pinned by tests/test_oracle_golden.py).

Parity bars:
* NVFP4 FP8-scale sweep: bit-exact per-block amax (the kernel keeps the reference kernel's fp32
  operation order).
* MSE multiplier sweep and AWQ-clip: the per-candidate losses are fp32 sums whose order the
  reference leaves to its reduction kernels (CPU and CUDA differ), so losses are compared with a
  relative tolerance and the chosen amax must equal the reference's wherever the reference's own
  losses separate the candidates by more than that tolerance ("near-tie" otherwise; every
  mismatch is checked to be one).
"""

import copy
import json
from functools import partial
from pathlib import Path

import pytest
import torch
import torch.nn as nn
from safetensors.torch import load_file

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"


def ops():
    from modelopt_amd import _ext

    return _ext.ops()


def same_bits(a, b):
    a, b = a.detach().cpu(), b.detach().cpu()
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    iv = {torch.float32: torch.int32, torch.float16: torch.int16, torch.bfloat16: torch.int16}[a.dtype]
    return bool((a.view(iv) == b.view(iv)).all())


def assert_best_or_near_tie(ours_idx, gold_idx, gold_losses, rel, max_frac=0.01, what=""):
    """ours_idx / gold_idx: chosen candidate per channel; gold_losses [K, C] (the reference's)."""
    ours_idx, gold_idx = ours_idx.reshape(-1).cpu(), gold_idx.reshape(-1).cpu()
    gl = gold_losses.reshape(gold_losses.shape[0], -1).cpu().double()
    bad = (ours_idx != gold_idx).nonzero().reshape(-1)
    assert bad.numel() <= max(1, int(max_frac * ours_idx.numel())), f"{what}: {bad.numel()} of {ours_idx.numel()} differ"
    for c in bad.tolist():
        lo, lg = gl[ours_idx[c], c], gl[gold_idx[c], c]
        assert lo <= lg * (1 + rel) + 1e-30, f"{what}: channel {c} picks {int(ours_idx[c])} (ref loss {lo}) over {int(gold_idx[c])} ({lg})"


def first_argmin(losses):
    return torch.argmin(losses.reshape(losses.shape[0], -1), dim=0)


# ---- NVFP4 FP8-scale sweep (nvfp4_fp8_sweep.py) -------------------------------------------------


@pytest.fixture(scope="module")
def mse_gold():
    return load_file(str(G / "mse.safetensors")), json.loads((G / "mse.json").read_text())


def test_nvfp4_sweep_matches_reference_kernel(gpu, mse_gold):
    from modelopt_amd.torch.quantization.calib.mse import fp8_scale_candidates

    t, meta = mse_gold
    assert torch.equal(fp8_scale_candidates("cpu"), t["sweep.candidates"])
    for name, m in meta["sweep"].items():
        x = t[f"sweep.{name}.x"].to(gpu)
        got = ops().nvfp4_fp8_scale_sweep(x, t[f"sweep.{name}.global_amax"].to(gpu), fp8_scale_candidates(gpu), m["block"])
        assert same_bits(got, t[f"sweep.{name}.best"]), name


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("nb,bs", [(1, 16), (257, 16), (4099, 16), (1000, 8), (333, 32)])
def test_nvfp4_sweep_vs_oracle(gpu, dtype, nb, bs):
    from modelopt_amd.torch.quantization.calib.mse import fp8_scale_candidates

    g = torch.Generator().manual_seed(nb * 7 + bs)
    x = (torch.randn(nb, bs, generator=g) * torch.logspace(-4, 2, nb)[:, None]).to(dtype)
    ga = x.float().abs().amax()
    got = ops().nvfp4_fp8_scale_sweep(x.to(gpu), ga.to(gpu), fp8_scale_candidates(gpu), bs)
    assert same_bits(got, R.nvfp4_fp8_scale_sweep(x, ga, bs))
    # an input that is not 16-byte aligned takes the scalar-load path
    buf = torch.zeros(nb * bs + 1, dtype=dtype)
    buf[1:] = x.reshape(-1)
    xu = buf.to(gpu)[1:].view(nb, bs)
    assert xu.data_ptr() % 16 != 0
    got_u = ops().nvfp4_fp8_scale_sweep(xu, ga.to(gpu), fp8_scale_candidates(gpu), bs)
    assert same_bits(got_u, got)


def test_nvfp4_sweep_rejects_bad_inputs(gpu):
    from modelopt_amd.torch.quantization.calib.mse import fp8_scale_candidates

    x = torch.randn(64, 16, device=gpu)
    with pytest.raises(ValueError):
        ops().nvfp4_fp8_scale_sweep(x, x.abs().amax(), fp8_scale_candidates(gpu), 12)
    with pytest.raises(ValueError):
        ops().nvfp4_fp8_scale_sweep(x.reshape(-1)[:1000], x.abs().amax(), fp8_scale_candidates(gpu), 16)
    with pytest.raises(RuntimeError):
        ops().nvfp4_fp8_scale_sweep(x.cpu(), x.abs().amax().cpu(), fp8_scale_candidates("cpu"), 16)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_nvfp4_mse_calibrator_fast_path_equals_reference_loop(gpu, dtype, monkeypatch):
    """The reference's own parity test (tests/gpu/.../test_nvfp4_fp8_sweep_kernel.py:93-116): the
    fused sweep and the 126-step loop over static_blockwise_fp4_fake_quant pick the same amax."""
    from modelopt_amd.torch.quantization.calib import NVFP4MSECalibrator
    from modelopt_amd.torch.quantization.tensor_quant import static_blockwise_fp4_fake_quant

    torch.manual_seed(0)
    x = torch.randn(1024, 16, device=gpu, dtype=dtype)
    pba = x.float().abs().amax(dim=-1)
    ga = pba.max()

    def run(fast):
        monkeypatch.setenv("MODELOPT_NVFP4_TRITON_SWEEP", "1" if fast else "0")
        cal = NVFP4MSECalibrator(amax=pba, axis=0, global_amax=ga,
                                 quant_func=lambda xx, a: static_blockwise_fp4_fake_quant(xx, a, ga))
        cal.collect(x)
        return cal.compute_amax()

    fast, loop = run(True), run(False)
    assert fast.dtype == torch.float32 and fast.shape == pba.shape
    assert torch.equal(fast, loop), f"{int((fast != loop).sum())} of {fast.numel()} blocks differ"
    cal = NVFP4MSECalibrator(amax=pba, axis=0, global_amax=ga, quant_func=None)
    monkeypatch.setenv("MODELOPT_NVFP4_TRITON_SWEEP", "1")
    cal.collect(x)
    with pytest.raises(RuntimeError, match="multi-collect"):
        cal.collect(x)
    cal.reset()
    cal.collect(x)
    assert torch.equal(cal.compute_amax(), fast)


# ---- MSE multiplier sweep (calib/mse.py MseCalibrator) ------------------------------------------


@pytest.mark.parametrize(
    "name,bits,shape,per_row,dtype",
    [("int8_rows", 8, (64, 96), True, torch.float32), ("int4_blocks", 4, (4096, 32), True, torch.bfloat16),
     ("int4_b128", 4, (777, 128), True, torch.float16), ("fp8_tensor", 0, (1, 70001), False, torch.float32),
     ("int8_long_rows", 8, (8, 5000), True, torch.bfloat16), ("fp8_rows", 0, (40, 300), True, torch.float32),
     ("int8_tensor_small", 8, (1, 100), False, torch.bfloat16)],
)
def test_mse_sweep_vs_oracle(gpu, name, bits, shape, per_row, dtype):
    g = torch.Generator().manual_seed(len(name))
    x = (torch.randn(shape, generator=g) * torch.logspace(-1, 0.5, shape[0])[:, None]).to(dtype)
    x.view(-1)[0] = 6.0
    amax = x.float().abs().amax(dim=1, keepdim=True) if per_row else x.float().abs().amax()
    amax = amax.to(dtype)
    cands = R.mse_candidates()
    if bits == 0:
        qf = lambda xx, a: R.fp8_eager(xx, a)  # noqa: E731
    else:
        qf = lambda xx, a: R.tensor_quant(xx, a, bits, False, False)  # noqa: E731
    ref_losses, ref_best = R.mse_sweep(x, amax, qf, 0 if per_row else None, cands)
    losses = ops().mse_sweep(x.to(gpu), amax.to(gpu), cands.to(gpu), bits, False, False, amax.dim() != 0)
    torch.testing.assert_close(losses.cpu(), ref_losses.reshape(losses.shape), rtol=2e-5, atol=0)
    assert_best_or_near_tie(first_argmin(losses), first_argmin(ref_losses), ref_losses, 2e-5, what=name)


def _golden_quantizer(m, w, gpu):
    from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig
    from modelopt_amd.torch.quantization.nn import TensorQuantizer

    qc = dict(m["cfg"])
    if isinstance(qc.get("num_bits"), list):
        qc["num_bits"] = tuple(qc["num_bits"])
    if m["block"]:
        qc["block_sizes"] = {-1: m["block"], "type": "static"}
    q = TensorQuantizer(QuantizerAttributeConfig(**qc)).to(gpu)
    q.enable_calib()
    q.disable_quant()
    q(w)
    q.load_calib_amax()
    q.disable_calib()
    q.enable_quant()
    return q


def test_mse_calibrator_matches_reference(gpu, mse_gold):
    from modelopt_amd.torch.quantization.calib import MseCalibrator
    from modelopt_amd.torch.quantization.model_calib import _mse_quant_func

    t, meta = mse_gold
    for name, m in meta["cal"].items():
        w = t[f"cal.{name}.w"].to(gpu)
        q = _golden_quantizer(m, w, gpu)
        assert same_bits(q._amax, t[f"cal.{name}.init_amax"]), name
        cal = MseCalibrator(amax=q._amax.clone(), axis=q._calibrator._axis, quant_func=partial(_mse_quant_func, quantizer=q))
        q._calibrator = cal
        q.enable_calib()
        q.disable_quant()
        q(w)
        losses = torch.stack([ls.reshape(-1) for ls in cal._losses_sum])
        gl = t[f"cal.{name}.losses"]
        torch.testing.assert_close(losses.cpu(), gl, rtol=2e-5, atol=0, msg=name)
        best = cal.compute_amax()
        assert best.dtype == t[f"cal.{name}.best"].dtype, name
        assert_best_or_near_tie(first_argmin(losses), first_argmin(gl), gl, 2e-5, what=name)
        if torch.equal(first_argmin(losses).cpu(), first_argmin(gl)):
            assert same_bits(best, t[f"cal.{name}.best"]), name


def _tiny_llama():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=32, max_position_embeddings=64)
    torch.manual_seed(40)
    return LlamaForCausalLM(cfg).eval()


@pytest.mark.parametrize("name,preset", [("int8", "INT8_DEFAULT_CFG"), ("fp8", "FP8_DEFAULT_CFG")])
def test_mse_calibrate_model_matches_reference(gpu, mse_gold, name, preset):
    import modelopt_amd.torch.quantization as mtq

    t, _ = mse_gold
    m = _tiny_llama().to(gpu)
    cfg = copy.deepcopy(getattr(mtq, preset))
    cfg["algorithm"] = {"method": "mse"}
    ids = t["model.calib_ids"].to(gpu)
    mtq.quantize(m, cfg, lambda mm: [mm(b) for b in ids])
    n = 0
    for k, v in t.items():
        if not k.startswith(f"model.{name}."):
            continue
        q = m.get_submodule(k[len(f"model.{name}."):])
        if k.endswith("weight_quantizer"):
            assert same_bits(q._amax, v), k  # weights: the MSE-searched amax
        else:
            torch.testing.assert_close(q._amax.cpu(), v, rtol=1e-5, atol=0)  # activations: max over GEMM outputs
        n += 1
    assert n >= 28


def test_nvfp4_mse_fp8_sweep_preset(gpu):
    """NVFP4_W4A4_WEIGHT_MSE_FP8_SWEEP_CFG end to end: every static NVFP4 weight's per-block amax
    is the oracle sweep of its blocks against its global amax."""
    import modelopt_amd.torch.quantization as mtq

    m = _tiny_llama().to(gpu).to(torch.bfloat16)
    ids = torch.randint(0, 32, (2, 2, 16), generator=torch.Generator().manual_seed(3)).to(gpu)
    mtq.quantize(m, mtq.NVFP4_W4A4_WEIGHT_MSE_FP8_SWEEP_CFG, lambda mm: [mm(b) for b in ids])
    n = 0
    for name, mod in m.named_modules():
        wq = getattr(mod, "weight_quantizer", None)
        if wq is None or not wq.is_enabled:
            continue
        w = mod.weight.detach().cpu()
        ref = R.nvfp4_fp8_scale_sweep(w.reshape(-1, 16), wq.global_amax.cpu(), 16)
        assert wq._amax.dtype == torch.float32
        assert same_bits(wq._amax.reshape(-1), ref), name
        n += 1
    assert n == 14
    with torch.no_grad():
        assert torch.isfinite(m(ids[0]).logits).all()


# ---- AWQ-clip (model_calib.py:1725-1940) --------------------------------------------------------


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("co,ci,bs,ntok", [(96, 256, 128, 64), (40, 64, 8, 70), (33, 100, 32, 5), (130, 512, 64, 127)])
def test_awq_clip_kernel_vs_oracle(gpu, dtype, co, ci, bs, ntok):
    g = torch.Generator().manual_seed(co + ci)
    w = (torch.randn(co, ci, generator=g) * 0.05).to(dtype)
    x = torch.randn(ntok, ci, generator=g).to(dtype)
    pad = (-ci) % bs
    wp = torch.nn.functional.pad(w, (0, pad))
    w_amax = wp.float().reshape(-1, bs).abs().amax(-1, keepdim=True).to(dtype)
    shrinks = R.awq_clip_shrinks()
    ref, ntk = R.awq_clip_block_losses(w, x, w_amax, shrinks, bs, max_tokens=1 << 30)
    assert ntk == ntok
    xs = torch.nn.functional.pad(x.float(), (0, pad)).contiguous()
    loss = torch.zeros(len(shrinks), co, (ci + pad) // bs, device=gpu)
    ops().awq_clip_search(wp.to(gpu), xs.to(gpu), w_amax.to(gpu), torch.tensor(shrinks), loss, bs, 4, False, False, True)
    rtol = 1e-4 if dtype == torch.float32 else 0.05
    got = loss.cpu()
    # bf16/f16: a product sum landing on a rounding boundary in one order and not the other moves a
    # dtype-rounded dot product by one ulp; such (block, shrink) losses are few and bounded
    rel = (got - ref).abs() / ref.abs().clamp_min(1e-30)
    frac_bad = float((rel > rtol).float().mean())
    assert frac_bad <= (0 if dtype == torch.float32 else 0.02), f"{frac_bad:.4f} of losses beyond rtol {rtol}"
    assert_best_or_near_tie(first_argmin(got), first_argmin(ref), ref, 0.05 if dtype != torch.float32 else 1e-4,
                            max_frac=0.03, what=str(dtype))
    # accumulate=False overwrites, accumulate=True adds
    ops().awq_clip_search(wp.to(gpu), xs.to(gpu), w_amax.to(gpu), torch.tensor(shrinks), loss, bs, 4, False, False, False)
    torch.testing.assert_close(loss.cpu(), got, rtol=0, atol=0)


class _ClipMLP(nn.Module):
    def __init__(self, f1=32, f2=16):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(16, f1, bias=False), nn.ReLU(), nn.Linear(f1, f2, bias=False),
                                 nn.ReLU(), nn.Linear(f2, 16, bias=False))

    def forward(self, x):
        return self.net(x)


@pytest.fixture(scope="module")
def clip_gold():
    return load_file(str(G / "awq_clip.safetensors")), json.loads((G / "awq_clip.json").read_text())


def _awq_cfg(mtq, method, block):
    cfg = copy.deepcopy(mtq.INT4_AWQ_CFG)
    for e in cfg["quant_cfg"]:
        if e.get("quantizer_name") == "*weight_quantizer":
            e["cfg"]["block_sizes"] = {-1: block, "type": "static"}
    cfg["algorithm"] = {"method": method, "debug": True}
    if method != "awq_clip":
        cfg["algorithm"]["alpha_step"] = 0.1
    return cfg


@pytest.mark.parametrize("name", ["mlp_clip", "mlp_full", "mlp_full_pad", "bf16_lin"])
def test_awq_clip_matches_reference(gpu, clip_gold, name):
    import modelopt_amd.torch.quantization as mtq

    t, meta = clip_gold
    m = meta[name]
    if name == "bf16_lin":
        model = nn.Sequential(nn.Linear(384, 192, bias=False)).to(torch.bfloat16)
    else:
        model = _ClipMLP(m["f1"], m["f2"])
    model.load_state_dict({k[len(name) + 4:]: v for k, v in t.items() if k.startswith(f"{name}.sd.")})
    model = model.to(gpu)
    data = [t[k].to(gpu) for k in sorted(k for k in t if k.startswith(f"{name}.data"))]
    mtq.quantize(model, _awq_cfg(mtq, m["method"], m["block"]), lambda mm: [mm(d.clone()) for d in data])
    bf16 = name == "bf16_lin"
    for n, lm in m["layers"].items():
        mod = model.get_submodule(n)
        h = mod.awq_clip
        assert h.shrinks == lm["shrinks"] and h.num_tokens == lm["num_tokens"], (name, n)
        full = m["method"] == "awq_full"  # awq_lite's scales agree to rtol 1e-4 (test_gpu_mtq)
        if full:
            torch.testing.assert_close(mod.weight.detach().cpu(), t[f"{name}.{n}.weight"], rtol=1e-4, atol=1e-6)
        assert h.w_amax.dtype == t[f"{name}.{n}.w_amax"].dtype
        torch.testing.assert_close(h.w_amax.cpu(), t[f"{name}.{n}.w_amax"], rtol=1e-4 if full else 0, atol=0)
        gl = t[f"{name}.{n}.losses"]
        got = h.loss_tensor.reshape(gl.shape).cpu()
        rel = (got - gl).abs() / gl.abs().clamp_min(1e-30)
        rtol = 0.05 if bf16 else (1e-3 if full else 1e-4)
        assert float((rel > rtol).float().mean()) <= (0.02 if bf16 else 0.0), (name, n)
        assert_best_or_near_tie(first_argmin(got), first_argmin(gl), gl, rtol, max_frac=0.03, what=f"{name}.{n}")
        if torch.equal(first_argmin(got), first_argmin(gl)) and m["method"] == "awq_clip":
            assert same_bits(h.best_clip_val, t[f"{name}.{n}.best_clip"]), (name, n)
    with torch.no_grad():
        out = model(t[f"{name}.test"].to(gpu).clone())
    tol = dict(rtol=0.05, atol=0.05) if bf16 else dict(rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(out.cpu().float(), t[f"{name}.out"].float(), **tol)
