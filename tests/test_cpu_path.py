"""The CPU execution path (BASELINE config C1: "INT8 per-tensor fake-quant on nn.Linear(1024,1024),
CPU eager reference path").

The reference registers its quantize op for ["cpu", "cuda"] (tensor_quant.py:252-256) and runs the
eager ATen sequences on CPU tensors.  The product's CPU kernels (csrc/mtq_cpu.cpp, C ABI
mtq_cpu_*) must give the same bits: checked here against the oracle (the restated ATen sequences,
pinned by the goldens) and, for C1 end to end, against the reference's own CPU run
(tests/golden/mtq_linear.safetensors, written by tests/golden/make_golden.py).  On the CPU the
GEMM is the same torch CPU GEMM the reference used, so outputs are bit-exact too.
"""

from pathlib import Path

import pytest
import torch
import torch.nn as nn
from safetensors.torch import load_file

from modelopt_amd import _ext
from oracle import ref_ops as R

G = Path(__file__).resolve().parent / "golden"
DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.float64]


def _same(a, b):
    iv = {torch.bfloat16: torch.int16, torch.float16: torch.int16, torch.float32: torch.int32,
          torch.float64: torch.int64}[a.dtype]
    nan = torch.isnan(a) & torch.isnan(b)
    return bool(((a.view(iv) == b.view(iv)) | nan).all())


def _x(dt, shape=(64, 300), seed=0):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(*shape, generator=g) * 3).to(dt)
    x[0, :5] = torch.tensor([float("nan"), float("inf"), -float("inf"), 0.0, -0.0]).to(dt)
    return x


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("bits,unsigned,narrow", [(8, False, False), (8, False, True), (4, False, False), (7, True, False)])
def test_int_qdq_per_tensor_and_axis(dt, bits, unsigned, narrow):
    ops = _ext.ops()
    x = _x(dt)
    if unsigned:
        x = x.abs()
    a = x[1:].float().abs().amax() * 0.7
    assert _same(ops.fake_tensor_quant(x, a, bits, unsigned, narrow), R.tensor_quant(x, a, bits, unsigned, narrow))
    ac = x.float().nan_to_num(0, 0, 0).abs().amax(dim=1, keepdim=True)
    ac[3] = 0  # zero amax -> zero output
    assert _same(ops.fake_tensor_quant_with_axis(x, ac.view(-1), 0, bits, unsigned, narrow),
                 R.tensor_quant(x, ac, bits, unsigned, narrow))
    assert _same(ops.quantize_op(x, ac, bits, 0, unsigned, narrow), R.tensor_quant(x, ac, bits, unsigned, narrow))
    y = x.clone()
    ops.fake_tensor_quant_(y, a, bits, unsigned, narrow)
    assert _same(y, R.tensor_quant(x, a, bits, unsigned, narrow))


@pytest.mark.parametrize("dt", DTYPES)
def test_fp8_qdq(dt):
    ops = _ext.ops()
    x = _x(dt)
    a = x[1:].float().abs().amax() * 0.7
    assert _same(ops.fake_e4m3fy(x, a), R.fp8_eager(x, a))
    ab = x.float().nan_to_num(0, 0, 0).abs().view(-1, 100).amax(dim=1, keepdim=True)
    assert _same(ops.quantize_op(x.view(-1, 100), ab, 8, 4, False, False), R.fp8_eager(x.view(-1, 100), ab))
    ac = x.float().nan_to_num(0, 0, 0).abs().amax(dim=0)
    assert _same(ops.fake_e4m3fy_with_axis(x, ac, 1), R.fp8_eager(x, ac.view(1, -1)))
    assert _same(ops.e4m3_cast(x), R.fp8_eager(x))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_fp8_and_int8_every_16bit_pattern(dt):
    ops = _ext.ops()
    allv = torch.arange(-32768, 32768, dtype=torch.int32).to(torch.int16).view(dt)
    assert _same(ops.e4m3_cast(allv), R.fp8_eager(allv))
    for amax in (1.0, 3.3, 448.0, 1e-30, 0.0, 1e5):
        t = torch.tensor(amax)
        assert _same(ops.fake_e4m3fy(allv, t), R.fp8_eager(allv, t)), amax
        assert _same(ops.fake_tensor_quant(allv, t, 8, False, False), R.tensor_quant(allv, t, 8, False, False)), amax


def test_amax_reductions():
    ops = _ext.ops()
    x = _x(torch.bfloat16)
    acc = torch.zeros(1)
    ops.amax_accumulate(x[1:], acc, 1, 1, x[1:].numel())
    assert acc.item() == x[1:].float().abs().max().item()
    acc = torch.zeros(300)
    ops.amax_accumulate(x[1:], acc, 63, 300, 1)
    assert torch.equal(acc, x[1:].float().abs().amax(0))
    acc = torch.zeros(64)
    ops.amax_accumulate(x, acc, 1, 64, 300)
    assert torch.equal(acc[1:], x[1:].float().abs().amax(1)) and torch.isnan(acc[0])
    # accumulation keeps the running max
    acc2 = torch.full((1,), 1e6)
    ops.amax_accumulate(x[1:], acc2, 1, 1, x[1:].numel())
    assert acc2.item() == 1e6


def test_c1_linear_int8_on_cpu():
    """C1 exactly as BASELINE.json states it, on the CPU: amax and outputs bit-exact with the
    reference's CPU run."""
    import modelopt_amd.torch.quantization as mtq

    t = load_file(str(G / "mtq_linear.safetensors"))
    m = nn.Linear(1024, 1024)
    m.load_state_dict({"weight": t["weight"], "bias": t["bias"]})
    calib = [t[f"calib{i}"] for i in range(4)]
    mtq.quantize(m, mtq.INT8_DEFAULT_CFG, lambda model: [model(c) for c in calib])
    assert torch.equal(m.input_quantizer.amax, t["input_amax"])
    assert torch.equal(m.weight_quantizer.amax, t["weight_amax"])
    with torch.no_grad():
        out = m(t["test"])
    assert torch.equal(out, t["out"])


def test_calibrate_under_inference_mode_on_cpu():
    """Calibration forwards run under torch.inference_mode() (inference tensors have no version
    counter; the reference's collect works there, so must ours)."""
    import modelopt_amd.torch.quantization as mtq

    t = load_file(str(G / "mtq_linear.safetensors"))
    m = nn.Linear(1024, 1024)
    m.load_state_dict({"weight": t["weight"], "bias": t["bias"]})
    calib = [t[f"calib{i}"] for i in range(4)]

    def loop(model):
        with torch.inference_mode():
            for c in calib:
                model(c)

    mtq.quantize(m, mtq.INT8_DEFAULT_CFG, loop)
    assert torch.equal(m.input_quantizer.amax, t["input_amax"])
    assert torch.equal(m.weight_quantizer.amax, t["weight_amax"])


def test_weight_written_through_data_is_recollected():
    """A weight changed through .data between two calibration passes (which does not bump
    _version) is reduced again: the "same tensor" skip does not outlive its pass."""
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.model_calib import max_calibrate

    m = nn.Linear(64, 64)
    mtq.quantize(m, mtq.INT8_DEFAULT_CFG, lambda mm: mm(torch.randn(4, 64)))
    a0 = m.weight_quantizer.amax.clone()
    m.weight.data.mul_(2.0)
    m.weight_quantizer.reset_amax()
    max_calibrate(m, lambda mm: mm(torch.randn(4, 64)))
    assert torch.equal(m.weight_quantizer.amax, a0 * 2)
