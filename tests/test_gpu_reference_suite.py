"""The reference's own GPU/unit test classes for the fake-quant path, restated against this build.

Each class / test names the reference test it restates (file:line, relative to the reference's
``tests/`` directory).  Same inputs, same assertions, with two systematic differences:

* the reference checks its CUDA ext against its own ATen path; here expected values come from the
  CPU oracle (``oracle/ref_ops.py``, pinned to the reference by tests/test_oracle_golden.py) or
  from the reference's tiny ``quant()`` INT restatement (_test_utils/torch/quantization/
  quant_utils.py:21-33, restated below), and compared bit-exactly where the reference uses
  ``atol=0``;
* tensors live on the ROCm device: this build has no CPU fake-quant path (by design -- the
  product fails loudly on CPU tensors), so the reference's ``device = "cpu"`` variants run on
  ``cuda`` here.
"""

from __future__ import annotations

import contextlib

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F
from pydantic import ValidationError

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu


def quant(x, amax, num_bits=8, fake=False, narrow_range=True):
    """The reference's test helper quant() (quant_utils.py:21-33), restated."""
    intmax = 2.0 ** (num_bits - 1) - 1.0
    intmin = -intmax if narrow_range else -intmax - 1
    scale = intmax / amax
    x_q = torch.clamp((x * scale).round_(), intmin, intmax)
    if fake:
        x_q /= scale
    return x_q


@pytest.fixture(scope="module")
def mtq(gpu):
    import modelopt_amd.torch.quantization as m

    return m


@pytest.fixture(scope="module")
def tq_mod(gpu):
    from modelopt_amd.torch.quantization import tensor_quant
    from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig
    from modelopt_amd.torch.quantization.nn.modules.tensor_quantizer import (
        SequentialQuantizer,
        TensorQuantizer,
    )

    class NS:
        pass

    ns = NS()
    ns.tensor_quant = tensor_quant
    ns.QAC = QuantizerAttributeConfig
    ns.TensorQuantizer = TensorQuantizer
    ns.SequentialQuantizer = SequentialQuantizer
    return ns


# ------------------------------------------------------------------------------------------------
# tests/_test_utils/torch/quantization/tensor_quant_common.py:26-137 (TensorQuantCommon /
# FakeTensorQuantTester), run by gpu/torch/quantization/test_tensor_quant_cuda.py:50
# ------------------------------------------------------------------------------------------------
class TestFakeTensorQuantCuda:
    def test_simple_run(self, tq_mod):
        x = torch.randn(2, 3, dtype=torch.float64).cuda() * 100
        tq_mod.tensor_quant.fake_tensor_quant(x, torch.max(torch.abs(x)), None, 7)

    def test_per_tensor_scale(self, tq_mod):
        x = torch.randn(31).cuda()
        ref = quant(x, torch.max(x.abs()), fake=True)
        out = tq_mod.tensor_quant.fake_tensor_quant(x, torch.max(torch.abs(x)))
        assert torch.allclose(ref, out)
        assert torch.equal(out.cpu(), R.tensor_quant(x.cpu(), x.abs().max().cpu()))

    def test_per_channel_scale(self, tq_mod):
        torch.manual_seed(123)
        x = torch.randn(3, 3, 6, 8).cuda()
        amax_x = 0.7 * torch.amax(x.abs(), dim=(1, 2, 3), keepdims=True)
        ref = quant(x, amax_x, fake=True)
        out = tq_mod.tensor_quant.fake_tensor_quant(x, amax_x)
        assert torch.allclose(out, ref)
        assert torch.equal(out.cpu(), R.tensor_quant(x.cpu(), amax_x.cpu()))

    def test_backward(self, tq_mod):
        x = torch.randn(3, 7, requires_grad=True, device="cuda")
        labels = torch.randint(6, (3,)).cuda()
        quant_x = tq_mod.tensor_quant.fake_tensor_quant(x, x.abs().max(), None, 7)
        float_quant_x = quant_x.float()
        x.retain_grad()
        float_quant_x.retain_grad()
        loss = nn.CrossEntropyLoss()(float_quant_x, labels)
        loss.backward()
        assert torch.allclose(float_quant_x.grad, x.grad)

    def test_unsigned(self, tq_mod):
        x = torch.randn(31).abs().cuda()
        ref = quant(x, torch.max(x.abs()), num_bits=9, fake=True)
        out = tq_mod.tensor_quant.fake_tensor_quant(x, torch.max(torch.abs(x)), None, 8, True)
        assert torch.allclose(out, ref)
        # the reference's CPU path raises TypeError("Negative values encountered ...")
        # (tensor_quant.py:612-613); the oracle restates it
        with pytest.raises(TypeError, match="Negative values encountered"):
            xn = torch.randn(3, 7)
            R.tensor_quant(xn, xn.abs().max(), 8, True)

    def test_clip_gradient(self, tq_mod):
        x = torch.randn(3, 7, requires_grad=True, device="cuda")
        x.retain_grad()
        amax = x.abs().max() / 2
        x_in_range = (-amax <= x) * (x <= amax)
        quant_x = tq_mod.tensor_quant.fake_tensor_quant(x, amax, None, 8)
        loss = torch.sum((quant_x - 0.5) ** 2)
        loss.backward()
        assert torch.equal(x.grad != 0, x_in_range)

    def test_full_range(self, tq_mod):
        x = torch.randn(31).abs().cuda()
        amax = torch.max(x.abs())
        ref = quant(x, amax, num_bits=9, fake=True, narrow_range=False)
        out = tq_mod.tensor_quant.fake_tensor_quant(x, torch.max(torch.abs(x)), None, 8, True, False)
        assert torch.allclose(out, ref)

    def test_overflow_fp16(self, tq_mod):
        # The reference passes (8, False) positionally into the (bias, num_bits) slots
        # (tensor_quant_common.py:131-136), i.e. num_bits = False = 0, which its CUDA kernel
        # feeds to `1 << (num_bits - 1)` (undefined behaviour).  The intent -- a tiny fp16 amax
        # whose scale 127 / 1e-4 overflows fp16 -- is tested with num_bits = 8; num_bits = 0 is
        # rejected by this build's C ABI with an error instead.
        x = torch.randn(31).cuda().half()
        amax = torch.tensor(1e-4).cuda().half()
        out = tq_mod.tensor_quant.fake_tensor_quant(x, amax, None, 8, False)
        assert not (torch.isinf(out).any() or torch.isnan(out).any())
        assert torch.equal(out.cpu(), R.tensor_quant(x.cpu(), amax.cpu(), 8, False))
        with pytest.raises(RuntimeError, match="invalid argument"):
            tq_mod.tensor_quant.fake_tensor_quant(x, amax, 8, False)


# ------------------------------------------------------------------------------------------------
# gpu/torch/quantization/test_tensor_quant_cuda.py:53-116 (TestCudaExt): the extension objects
# ------------------------------------------------------------------------------------------------
class TestCudaExt:
    @pytest.fixture(scope="class")
    def ext(self, gpu):
        from modelopt_amd.torch.quantization.extensions import get_cuda_ext

        e = get_cuda_ext(raise_if_failed=True)
        assert e is not None
        return e

    @pytest.mark.parametrize("num_bits", [3, 4, 5, 7, 8, 11])
    @pytest.mark.parametrize("unsigned", [True, False])
    def test_cuda_ext_num_bits(self, ext, tq_mod, num_bits, unsigned):
        x = torch.randn(31).cuda()
        if unsigned:
            x = x.abs()
        a = torch.max(torch.abs(x))
        out = ext.fake_tensor_quant(x, a, num_bits, unsigned)
        assert torch.equal(out, tq_mod.tensor_quant.fake_tensor_quant(x, a, None, num_bits, unsigned))
        assert torch.equal(out.cpu(), R.tensor_quant(x.cpu(), a.cpu(), num_bits, unsigned))

    @pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
    def test_cuda_ext_dtype(self, ext, dtype):
        x = torch.randn(31).cuda().to(dtype)
        a = torch.max(torch.abs(x))
        out = ext.fake_tensor_quant(x, a).float()
        assert torch.equal(out.cpu(), R.tensor_quant(x.cpu(), a.cpu()).float())

    @pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
    @pytest.mark.parametrize("num_bits", [3, 4, 5, 7, 8, 11])
    @pytest.mark.parametrize("unsigned", [True, False])
    def test_cuda_ext_with_axis(self, ext, dtype, num_bits, unsigned):
        x = torch.randn(3, 4, 5, 6).cuda().to(dtype)
        amax = torch.tensor([0.8, 0.9, 0.7, 0.6]).cuda()
        if unsigned:
            x = x.abs()
        out = ext.fake_tensor_quant_with_axis(x, amax, 1, num_bits, unsigned).float()
        ref = R.tensor_quant(x.cpu(), amax.view(1, -1, 1, 1).cpu(), num_bits, unsigned).float()
        assert torch.equal(out.cpu(), ref)

    @pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
    def test_cuda_ext_inplace(self, ext, dtype):
        torch.manual_seed(1234)
        x = torch.randn(31).cuda().to(dtype)
        ref = quant(x, torch.max(x.abs()), fake=True)
        exact = R.tensor_quant(x.cpu(), x.abs().max().cpu())
        ext.fake_tensor_quant_(x, torch.max(torch.abs(x)))
        atol = {torch.bfloat16: 1e-1, torch.float16: 1e-3}.get(dtype, 1e-8)
        assert torch.allclose(x, ref, atol=atol)
        assert torch.equal(x.cpu(), exact)

    def test_cuda_ext_tiny_amax(self, ext):
        x = torch.rand(2, 3, 4).cuda()
        amax = torch.tensor([1.0, 1.0e-26, 1.0]).cuda().unsqueeze(-1).unsqueeze(1)
        out = ext.fake_tensor_quant_with_axis(x, amax, axis=1)
        assert out[:, 1, :].sum() == 0


# ------------------------------------------------------------------------------------------------
# gpu/torch/quantization/test_tensor_quant_cuda.py:119-182 (TestScaledE4M3); fp8_eager = oracle
# ------------------------------------------------------------------------------------------------
class TestScaledE4M3:
    def test_e4m3_no_scale(self, tq_mod):
        x = torch.randn(4, 4, device="cuda")
        ref = R.fp8_eager(x.cpu(), torch.tensor(448.0))
        out = tq_mod.tensor_quant.scaled_e4m3(x, None, None, 4, 3)
        assert torch.allclose(out.cpu(), ref, atol=1e-4, rtol=1e-4)

    @pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
    def test_with_amax(self, tq_mod, dtype):
        from modelopt_amd.torch.quantization.utils import core_utils as quant_utils

        x = torch.randn(4, 4, device="cuda", dtype=dtype)
        amax = quant_utils.reduce_amax(x, axis=None, keepdims=True)
        out = tq_mod.tensor_quant.scaled_e4m3(x, amax, None, 4, 3)
        assert torch.equal(out.cpu(), R.fp8_eager(x.cpu(), amax.cpu()))

    def test_e4m3_incontiguous(self, tq_mod):
        x = torch.randn(4, 4).cuda().transpose(1, 0)
        assert not x.is_contiguous()
        ref = R.fp8_eager(x.cpu(), torch.tensor(448.0))
        out = tq_mod.tensor_quant.scaled_e4m3(x, None, None, 4, 3)
        assert torch.allclose(out.cpu(), ref, atol=1e-4, rtol=1e-4)

    def test_backward(self, tq_mod):
        x = torch.randn(3, 7, requires_grad=True, device="cuda")
        labels = torch.randint(6, (3,)).cuda()
        quant_x = tq_mod.tensor_quant.scaled_e4m3(x, None, None, 4, 3)
        x.retain_grad()
        quant_x.retain_grad()
        nn.CrossEntropyLoss()(quant_x, labels).backward()
        assert torch.allclose(quant_x.grad, x.grad)

    @pytest.mark.parametrize("axis", [0, 1, 2])
    def test_e4m3_per_channel(self, tq_mod, axis):
        x = torch.randn(4, 4, 4).cuda()
        amax = x.abs().amax(dim=[ax for ax in range(x.ndim) if ax != axis], keepdim=True)
        out = tq_mod.tensor_quant.scaled_e4m3(x, amax, None, 4, 3)
        assert torch.equal(out.cpu(), R.fp8_eager(x.cpu(), amax.cpu()))

    def test_zero_amax_is_finite(self, tq_mod):
        x = torch.randn(4, 4, device="cuda")
        out = tq_mod.tensor_quant.scaled_e4m3(x, torch.zeros((1,), device="cuda"), None, 4, 3)
        assert torch.isfinite(out).all()

    def test_zero_amax_per_channel_is_finite(self, tq_mod):
        x = torch.randn(2, 3, 4, device="cuda")
        amax = torch.tensor([1.0, 0.0, 1.0], device="cuda").view(1, 3, 1)
        out = tq_mod.tensor_quant.scaled_e4m3(x, amax, None, 4, 3)
        assert torch.isfinite(out).all()


# ------------------------------------------------------------------------------------------------
# gpu/torch/quantization/test_tensor_quant_cuda.py:205-262 (Testfp4.test_cuda_ext_fp4): E2M1 KATs
# through fused_amax_convert with E4M3 block scales and a global amax
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("block_size", [8, 16, 32])
def test_cuda_ext_fp4(gpu, dtype, block_size):
    from modelopt_amd.torch.quantization.extensions import get_cuda_ext_mx
    from modelopt_amd.torch.quantization.tensor_quant import mx_format_map

    mx = get_cuda_ext_mx(raise_if_failed=True)
    sign = torch.randint(0, 2, (1, 8)).cuda() * 2 - 1

    def check(test_in, test_out):
        inputs = torch.concat((test_in,) * (block_size // 8), dim=-1).to(dtype)
        expected = torch.concat((test_out,) * (block_size // 8), dim=-1).to(dtype)
        out = mx.fused_amax_convert(
            inputs, 16, getattr(mx.Types, mx_format_map[(2, 1)]), getattr(mx.Types, mx_format_map[(4, 3)]),
            inputs.abs().amax().float(),
        )
        assert torch.allclose(out.float(), expected.float())

    table = torch.tensor([[0, 0.5, 1, 1.5, 2, 3, 4, 6]]).cuda()
    check(table * sign, table * sign)
    bnd = torch.tensor([[0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5, 6]]).cuda()
    check(bnd * sign, torch.tensor([[0.0, 1, 1, 2, 2, 4, 4, 6]]).cuda() * sign)
    below = bnd.clone()
    below[:, :-1] -= 0.1
    check(below * sign, torch.tensor([[0.0, 0.5, 1, 1.5, 2, 3, 4, 6]]).cuda() * sign)
    above = bnd.clone()
    above[:, :-1] += 0.1
    check(above * sign, torch.tensor([[0.5, 1, 1.5, 2, 3, 4, 6, 6]]).cuda() * sign)


# ------------------------------------------------------------------------------------------------
# _test_utils/torch/quantization/tensor_quantizer_common.py:34-477 (TensorQuantizerTester), run by
# gpu/torch/quantization/test_tensor_quantizer_cuda.py:33 with device = "cuda"
# ------------------------------------------------------------------------------------------------
class TestTensorQuantizerCuda:
    def test_simple_run(self, tq_mod):
        x = torch.randn(3, 7).cuda()
        fn = tq_mod.tensor_quant.fake_tensor_quant(x, torch.max(torch.abs(x)), None)
        assert torch.equal(fn, tq_mod.TensorQuantizer()(x))

    def test_per_tensor_scale(self, tq_mod):
        x = torch.randn(31).cuda()
        ref = quant(x, torch.max(torch.abs(x)), fake=True)
        q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8))
        assert torch.allclose(q(x), ref)

    def test_per_channel_scale(self, tq_mod):
        x = torch.randn(5, 5, 4, 8).cuda()
        amax_x = torch.amax(x.abs(), axis=(1, 2, 3), keepdims=True)
        ref = quant(x, amax_x, fake=True)
        q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, axis=(0))).cuda()
        assert torch.allclose(q(x), ref, rtol=1e-2)

    def test_disable(self, tq_mod):
        x = torch.randn(3, 7).cuda()
        q = tq_mod.TensorQuantizer(tq_mod.QAC(enable=False)).cuda()
        assert torch.equal(x, q(x))

    def test_state_loading(self, tq_mod):
        amax = [3.14, 2.718]
        q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=(4, 3)), amax=amax).cuda()
        q.load_state_dict(q.state_dict())
        assert torch.allclose(q.amax, torch.tensor(amax).cuda())

    def test_properties(self, tq_mod):
        q1 = tq_mod.TensorQuantizer(tq_mod.QAC(), amax=3.14).cuda()
        q1.amax = 0.577
        assert q1.amax == torch.tensor(0.577).cuda()
        assert q1.step_size == 0.577 / 127.0
        q2 = tq_mod.TensorQuantizer(tq_mod.QAC()).cuda()
        amax = torch.tensor([3.142, 2.718]).cuda()
        q2.amax = amax
        assert torch.allclose(q2.amax, amax)
        assert tq_mod.TensorQuantizer(tq_mod.QAC()).amax is None

    def test_init_calib(self, tq_mod):
        q = tq_mod.TensorQuantizer(tq_mod.QAC(axis=(0, 1)), if_calib=True, if_quant=False).cuda()
        q(torch.rand(7, 6, 7, 7).cuda())
        q.load_calib_amax()
        assert q.amax.numel() == 7 * 6

    def test_max_calib(self, tq_mod):
        from modelopt_amd.torch.quantization.utils import core_utils as quant_utils

        q = tq_mod.TensorQuantizer(tq_mod.QAC(axis=0)).cuda()
        q.enable_calib()
        with pytest.raises(RuntimeError, match="Calibrator returned None"):
            q.load_calib_amax()
        x1, x2 = torch.rand(7, 6, 7, 7).cuda(), torch.rand(7, 6, 7, 7).cuda()
        q(x1)
        q(x2)
        q.disable_calib()
        g = torch.max(
            quant_utils.reduce_amax(x1, axis=(1, 2, 3), keepdims=True),
            quant_utils.reduce_amax(x2, axis=(1, 2, 3), keepdims=True),
        )
        assert torch.equal(q._calibrator.compute_amax(), g)
        q.load_calib_amax()
        assert torch.equal(q.amax, g)
        want = torch.max(R.reduce_amax(x1.cpu(), axis=(1, 2, 3)), R.reduce_amax(x2.cpu(), axis=(1, 2, 3)))
        assert torch.equal(q.amax.cpu(), want)

    def test_entropy_and_percentile_calib(self, tq_mod):
        q = tq_mod.TensorQuantizer(tq_mod.QAC(calibrator="histogram"), if_calib=True, if_quant=False).cuda()
        q._calibrator._num_bins = 512
        x1, x2 = torch.rand(3, 6, 7, 7).cuda(), torch.rand(3, 6, 7, 7).cuda()
        q(x1)
        q(x2)
        q.load_calib_amax("entropy")
        assert torch.equal(q._calibrator.compute_amax("entropy"), q.amax)
        q._calibrator.reset()
        q(x1)
        q(x2)
        q.load_calib_amax("percentile", percentile=99.99)
        assert torch.equal(q._calibrator.compute_amax("percentile", percentile=99.99), q.amax)

    def test_setters(self, tq_mod):
        q = tq_mod.TensorQuantizer()
        q.num_bits = 7
        q.unsigned = True
        assert q.num_bits == 7
        assert q.unsigned

    def test_pre_quant_scale(self, tq_mod):
        cfg = tq_mod.QAC(axis=1, num_bits=8)
        q = tq_mod.TensorQuantizer(cfg, amax=127.0).cuda()
        q2 = tq_mod.TensorQuantizer(cfg, amax=127.0).cuda()
        inputs = torch.Tensor([[0, 0.4, 1.1, 2.0]]).cuda()
        assert torch.allclose(q(inputs), torch.Tensor([[0, 0, 1, 2]]).cuda())
        q.pre_quant_scale = 2.0
        assert torch.allclose(q(inputs), torch.Tensor([[0, 1, 2, 4]]).cuda())
        q2.pre_quant_scale = torch.Tensor([[1.0, 2.0, 3.0, 4.0]]).cuda()
        assert torch.allclose(q2(inputs), torch.Tensor([[0, 1, 3, 8]]).cuda())

    def test_set_from_attribute_config(self, tq_mod):
        q = tq_mod.TensorQuantizer()
        q.set_from_attribute_config({"num_bits": 4})
        assert q.num_bits == 4
        q.set_from_attribute_config({"axis": -1})
        assert q.axis == -1
        q.set_from_attribute_config({"enable": False})
        assert q._disabled

    def test_use_constant_amax(self, tq_mod):
        x = torch.randn(4, 8).cuda()
        q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, use_constant_amax=True)).cuda()
        assert q._use_constant_amax is True
        a = q._get_amax(x)
        assert a.item() == torch.finfo(torch.float8_e4m3fn).max
        assert a.device == x.device
        assert q(x).shape == x.shape

    def test_use_constant_amax_skips_calibration(self, tq_mod):
        from modelopt_amd.torch.quantization.model_calib import enable_stats_collection, finish_stats_collection

        model = nn.ModuleDict({
            "tq_const": tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, use_constant_amax=True)),
            "tq_calib": tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8)),
        }).cuda()
        enable_stats_collection(model)
        assert not model["tq_const"]._disabled
        assert not model["tq_const"]._if_calib and not model["tq_const"]._if_quant
        assert not model["tq_calib"]._disabled
        assert model["tq_calib"]._if_calib and not model["tq_calib"]._if_quant
        finish_stats_collection(model)
        assert not model["tq_const"]._disabled and model["tq_const"]._if_quant

    def test_constant_amax_registers_amax(self, tq_mod):
        nv = {"num_bits": (2, 1), "block_sizes": {-1: 16, "type": "dynamic", "scale_bits": (4, 3)}}
        q = tq_mod.TensorQuantizer(tq_mod.QAC(**nv, constant_amax=2688.0)).cuda()
        assert q._constant_amax == 2688.0
        assert hasattr(q, "_amax") and float(q._amax) == 2688.0
        q0 = tq_mod.TensorQuantizer(tq_mod.QAC(**nv)).cuda()
        assert q0._constant_amax is None and not hasattr(q0, "_amax")

    def test_constant_amax_nvfp4_input_scale(self, tq_mod):
        from modelopt_amd.torch.export.quant_utils import get_activation_scaling_factor

        nv = {"num_bits": (2, 1), "block_sizes": {-1: 16, "type": "dynamic", "scale_bits": (4, 3)}}
        q = tq_mod.TensorQuantizer(tq_mod.QAC(**nv, constant_amax=2688.0)).cuda()
        m = nn.Module()
        m.input_quantizer = q
        s = get_activation_scaling_factor(m)
        assert torch.allclose(s.float(), torch.ones_like(s.float()))

    def test_constant_amax_skips_calibration(self, tq_mod):
        from modelopt_amd.torch.quantization.model_calib import enable_stats_collection, finish_stats_collection

        nv = {"num_bits": (2, 1), "block_sizes": {-1: 16, "type": "dynamic", "scale_bits": (4, 3)}}
        model = nn.ModuleDict({
            "tq_const": tq_mod.TensorQuantizer(tq_mod.QAC(**nv, constant_amax=2688.0)),
            "tq_calib": tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8)),
        }).cuda()
        enable_stats_collection(model)
        assert not model["tq_const"]._if_calib and not model["tq_const"]._if_quant
        assert float(model["tq_const"]._amax) == 2688.0
        finish_stats_collection(model)
        assert model["tq_const"]._if_quant and float(model["tq_const"]._amax) == 2688.0

    def test_constant_amax_must_be_positive(self, tq_mod):
        for v in (-1.0, 0.0):
            with pytest.raises(Exception, match="constant_amax must be a positive value"):
                tq_mod.QAC(num_bits=(2, 1), constant_amax=v)

    def test_constant_amax_mutually_exclusive_with_use_constant_amax(self, tq_mod):
        with pytest.raises(Exception, match="mutually exclusive"):
            tq_mod.QAC(num_bits=8, use_constant_amax=True, constant_amax=2688.0)

    def test_modelopt_state(self, tq_mod):
        ref = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=4), amax=10.0).cuda()
        test = tq_mod.TensorQuantizer(tq_mod.QAC())
        state = ref.get_modelopt_state()
        for k in ref._get_properties_for_modelopt_state():
            assert k in state
            assert state[k] == getattr(ref, k)
        assert "_pytorch_state_metadata" in state
        assert "_amax" not in state and "_amax" in state["_pytorch_state_metadata"]["buffers"]
        test.set_from_modelopt_state(state)
        test.load_state_dict(ref.state_dict())
        test.cuda()
        x = torch.randn(10, 10).cuda()
        assert torch.equal(ref(x), test(x))

    def test_amax_export(self, tq_mod):
        a = torch.randn(4, 6, 8).cuda()
        for bs, last in ((4, 2), (8, 1)):
            q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=4, block_sizes={-1: bs}))
            assert not hasattr(q, "_amax_shape_for_export")
            q(a)
            q.enable_calib()
            q(a)
            q.load_calib_amax()
            amax = q.export_amax()
            assert getattr(q, "_amax_shape_for_export", None) == (4, 6, -1)
            assert amax.shape == (4, 6, last), amax.shape
        q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=4, axis=0))
        q.enable_calib()
        q(a)
        q.load_calib_amax()
        amax = q.export_amax()
        assert not hasattr(q, "_amax_shape_for_export")
        assert amax.shape == (4,), amax.shape
        q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=4))
        q.enable_calib()
        q(a)
        q.load_calib_amax()
        assert q.export_amax().shape == (1,)

    def test_save_restore(self, tq_mod):
        ref = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=4, axis=0))
        ref.enable_calib()
        ref(torch.randn(4, 6, 8).cuda())
        ref(torch.randn(4, 6, 8).cuda())
        ref.load_calib_amax()
        ref.disable_calib()
        state = ref.get_modelopt_state()
        test = tq_mod.TensorQuantizer(tq_mod.QAC())
        test.set_from_modelopt_state(state)
        test.load_state_dict(ref.state_dict())
        inp = torch.randn(4, 6, 8).cuda()
        assert torch.equal(ref(inp), test(inp))

    def test_backward(self, tq_mod):
        x = torch.randn(3, 7, requires_grad=True, device="cuda")
        tq_mod.TensorQuantizer()(x).sum().backward()

    def test_block_sizes_axis(self, tq_mod):
        test_w = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, block_sizes={1: None}))
        ref_w = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, axis=0))
        test_i = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, block_sizes={0: None, 1: None}))
        ref_i = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, axis=-1))
        inp = torch.randn(1, 2, 3).cuda()
        w = torch.randn(3, 3).cuda()
        assert torch.equal(test_w(w), ref_w(w))
        assert torch.equal(test_i(inp), ref_i(inp))


# ------------------------------------------------------------------------------------------------
# _test_utils/torch/quantization/tensor_quantizer_common.py:480-582 (BlockQuantTester)
# ------------------------------------------------------------------------------------------------
class TestBlockQuantCuda:
    def test_simple(self, tq_mod):
        a = torch.randn(8, 4).cuda()
        amax_ref = a.view(-1, 2).abs().amax(dim=-1, keepdim=True)
        ref = R.tensor_quant(a.view(-1, 2).cpu(), amax_ref.cpu(), 8, False, False).view_as(a)
        for bs in ({-1: 2}, {1: 2}):
            q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, block_sizes=bs))
            q.enable_calib()
            out = q(a)
            q.load_calib_amax()
            assert torch.equal(q.amax, amax_ref)
            assert torch.equal(out.cpu(), ref)

    def test_complex(self, tq_mod):
        a = torch.randn(2, 6, 4).cuda()
        a_max = a.reshape(2, 2, 3, 2, 2).abs().amax(dim=(2, 4), keepdim=True)
        ref = R.tensor_quant(a.reshape(2, 2, 3, 2, 2).cpu(), a_max.cpu(), 8, False, False).view_as(a)
        for bs in ({-1: 2, 1: 3}, {1: 3, 2: 2}):
            q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, block_sizes=bs))
            assert torch.equal(q(a).cpu(), ref)

    def test_simple_padding(self, tq_mod):
        a = torch.randn(3, 4, 5).cuda()
        a_padded = F.pad(a, (0, 1), mode="constant", value=0)
        amax = a_padded.view(-1, 2).abs().amax(dim=-1, keepdim=True)
        ref = R.tensor_quant(a_padded.view(-1, 2).cpu(), amax.cpu(), 8, False, False).view_as(a_padded)[:, :, :5]
        for bs in ({-1: 2}, {2: 2}):
            q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, block_sizes=bs))
            q.enable_calib()
            out = q(a)
            q.load_calib_amax()
            assert torch.equal(q.amax, amax)
            assert torch.equal(out.cpu(), ref)

    def test_complex_padding(self, tq_mod):
        a = torch.randn(2, 10, 5).cuda()
        a_padded = F.pad(a, (0, 1, 0, 2), mode="constant", value=0)
        amax = a_padded.view(2, 4, 3, 3, 2).abs().amax(dim=(2, 4), keepdim=True)
        ref = R.tensor_quant(a_padded.view(2, 4, 3, 3, 2).cpu(), amax.cpu(), 8, False, False).view_as(a_padded)[:, :10, :5]
        q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, block_sizes={-1: 2, 1: 3}))
        q.enable_calib()
        out = q(a)
        q.load_calib_amax()
        assert torch.equal(amax, q.amax)
        assert torch.equal(out.cpu(), ref)
        q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=8, block_sizes={1: 3, 2: 2}))
        assert torch.equal(q(a).cpu(), ref)


# ------------------------------------------------------------------------------------------------
# _test_utils/torch/quantization/tensor_quantizer_common.py:585-646 (SequentialQuantizerTester)
# ------------------------------------------------------------------------------------------------
class TestSequentialQuantizer:
    def test_sequential_quantizer(self, tq_mod):
        TQ, QAC = tq_mod.TensorQuantizer, tq_mod.QAC
        nq = tq_mod.SequentialQuantizer(TQ(QAC()), TQ(QAC()), TQ(QAC()))
        tqs = [TQ() for _ in range(3)]
        for qs in (nq, tqs):
            qs[0].set_from_attribute_config({"num_bits": 4})
            qs[1].set_from_attribute_config({"block_sizes": {-1: 4}})
            qs[2].set_from_attribute_config({"enable": False})
        x = torch.randn(2, 16).cuda()
        ref = x
        for q in tqs:
            ref = q(ref)
        assert torch.equal(ref, nq(x))

    def test_replace_sequential_quantizer(self, tq_mod):
        from modelopt_amd.torch.quantization.nn import QuantLinear

        TQ, QAC = tq_mod.TensorQuantizer, tq_mod.QAC
        model = nn.Module()
        model.model = nn.Sequential(QuantLinear(4, 4), nn.ReLU())
        model.model[0].weight_quantizer = tq_mod.SequentialQuantizer(TQ(QAC()), TQ(QAC()))
        sq = model.model[0].weight_quantizer
        with tq_mod.SequentialQuantizer.convert_to_single_quantizer(model):
            for _, module in model.model.named_modules():
                assert not isinstance(module, tq_mod.SequentialQuantizer)
        assert model.model[0].weight_quantizer is sq
        assert not hasattr(model.model[0], "_original_weight_quantizer")

    def test_sequential_quantizer_attribute(self, tq_mod):
        from modelopt_amd.torch.quantization.model_calib import max_calibrate

        TQ, QAC = tq_mod.TensorQuantizer, tq_mod.QAC
        sq = tq_mod.SequentialQuantizer(TQ(QAC()), TQ(QAC())).cuda()
        sq.disable()
        assert sq[0].is_enabled is False and sq[1].is_enabled is False
        sq.enable()
        assert sq[0].is_enabled is True and sq[1].is_enabled is True
        max_calibrate(sq, lambda m: m(torch.randn(1, 4).cuda()))
        sq.reset_amax()
        assert sq[0].amax is None and sq[1].amax is None
        assert sq.fake_quant is True
        sq[0]._fake_quant = False
        assert sq.fake_quant is False and sq[1]._fake_quant is True


# ------------------------------------------------------------------------------------------------
# gpu/torch/quantization/test_tensor_quantizer_cuda.py:41-121 (E4M3 quantizer, FP4 quantizer)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize(("E", "M", "axis"), [(5, 2, None), (4, 3, None), (4, 3, 1), (7, 3, None)])
def test_tensor_quantizer_e4m3(tq_mod, E, M, axis):  # noqa: N803
    expect_error = E != 4 or M != 3
    with pytest.raises(ValidationError) if expect_error else contextlib.nullcontext():
        q = tq_mod.TensorQuantizer(tq_mod.QAC(num_bits=(E, M), axis=axis)).cuda()
        x = torch.rand(3, 6, 7, 7).cuda()
        out = q(x)
        ref = tq_mod.tensor_quant.scaled_e4m3(x, q._get_amax(x), None, E, M)
        assert torch.equal(out, ref)
        assert torch.equal(out.cpu(), R.fp8_eager(x.cpu(), q._get_amax(x).cpu()))


def test_tensor_quantizer_fp4(tq_mod):
    q = tq_mod.TensorQuantizer(
        tq_mod.QAC(num_bits=(2, 1), block_sizes={-1: 16, "type": "dynamic", "scale_bits": (4, 3)})
    ).cuda()
    x = torch.rand(2, 1, 16).cuda()
    out = q(x)
    ref = tq_mod.tensor_quant.dynamic_block_quant(x, 16, x.abs().amax(), None, (2, 1), (4, 3))
    assert torch.equal(out, ref)
    assert q._get_amax(x) == x.abs().amax()


@pytest.mark.parametrize("pass_through_bwd", [True, False])
def test_tensor_quantizer_fp4_backward(tq_mod, pass_through_bwd):
    q = tq_mod.TensorQuantizer(
        tq_mod.QAC(num_bits=(2, 1), block_sizes={-1: 16, "type": "dynamic", "scale_bits": (4, 3)},
                   pass_through_bwd=pass_through_bwd)
    ).cuda()
    x = torch.rand(2, 1, 16).cuda()
    with torch.no_grad():
        q.amax = torch.median(x.abs())
    x.requires_grad = True
    q(x).sum().backward()
    want = torch.ones_like(x.grad) if pass_through_bwd else torch.ones_like(x.grad) * (x.abs() <= q.amax)
    assert torch.equal(x.grad, want)


def test_tensor_quantizer_fp4_non_contiguous_input(tq_mod):
    contiguous = torch.ones(2, 16).cuda()
    large = torch.ones(2, 32).cuda()
    large[:, :16] = torch.randn(2, 16).cuda()
    non_contiguous = large[:, 16:]
    assert torch.equal(contiguous, non_contiguous) and not non_contiguous.is_contiguous()
    q = tq_mod.TensorQuantizer(
        tq_mod.QAC(num_bits=(2, 1), block_sizes={-1: 16, "type": "dynamic", "scale_bits": (4, 3)},
                   axis=None, enable=True)
    ).cuda()
    assert torch.equal(q(contiguous), q(non_contiguous))


# ------------------------------------------------------------------------------------------------
# unit/torch/quantization/test_quant_linear.py:31-222 (TestQuantLinear).  The expected operands
# come from the oracle; the GEMM is the same F.linear on the device, so equality is exact.
# ------------------------------------------------------------------------------------------------
class TestQuantLinear:
    @staticmethod
    def qdq(x, amax, num_bits=8):
        return R.tensor_quant(x.detach().cpu(), amax.detach().cpu(), num_bits).cuda()

    def test_weight_fake_per_tensor(self, tq_mod):
        from modelopt_amd.torch.quantization.nn.modules import quant_linear

        m = quant_linear.QuantLinear(2, 2, bias=False, quant_desc_weight=tq_mod.QAC(axis=None)).cuda()
        m.input_quantizer.disable()
        x = torch.randn(2, 2).cuda()
        w = m.weight.clone()
        assert torch.equal(F.linear(x, self.qdq(w, w.abs().max())), m(x))

    def test_weight_fake_per_channel(self, tq_mod):
        from modelopt_amd.torch.quantization.nn.modules import quant_linear

        m = quant_linear.QuantLinear(
            3, 5, bias=False, quant_desc_weight=tq_mod.tensor_quant.QUANT_DESC_8BIT_LINEAR_WEIGHT_PER_ROW
        ).cuda()
        m.input_quantizer.disable()
        x = torch.randn(32, 3).cuda()
        w = m.weight.clone()
        amax = w.abs().amax(dim=1, keepdim=True)
        assert torch.equal(F.linear(x, self.qdq(w, amax)), m(x))

    def test_input_fake_per_tensor(self, tq_mod):
        from modelopt_amd.torch.quantization.nn.modules import quant_linear

        m = quant_linear.QuantLinear(3, 5, bias=False).cuda()
        m.weight_quantizer.disable()
        x = torch.randn(32, 3).cuda()
        assert torch.equal(F.linear(self.qdq(x, x.abs().max()), m.weight), m(x))

    def test_fake_quant_per_tensor(self, tq_mod):
        from modelopt_amd.torch.quantization.nn.modules import quant_linear

        m = quant_linear.QuantLinear(3, 5, bias=False, quant_desc_weight=tq_mod.QAC()).cuda()
        x = torch.randn(32, 3).cuda()
        w = m.weight.clone()
        assert torch.equal(F.linear(self.qdq(x, x.abs().max()), self.qdq(w, w.abs().max())), m(x))

    def test_fake_quant_per_tensor_with_bias(self, tq_mod):
        from modelopt_amd.torch.quantization.nn.modules import quant_linear

        m = quant_linear.QuantLinear(3, 5, bias=False, quant_desc_weight=tq_mod.QAC()).cuda()
        x = torch.randn(32, 17, 93, 3).cuda()
        w = m.weight.clone()
        ref = F.linear(self.qdq(x, x.abs().max()), self.qdq(w, w.abs().max()), bias=m.bias)
        assert torch.equal(ref, m(x))

    def test_fake_quant_per_channel(self, tq_mod):
        from modelopt_amd.torch.quantization.nn.modules import quant_linear

        m = quant_linear.QuantLinear(
            3, 5, bias=False, quant_desc_weight=tq_mod.tensor_quant.QUANT_DESC_8BIT_LINEAR_WEIGHT_PER_ROW
        ).cuda()
        x = torch.randn(2, 3).cuda()
        w = m.weight.clone()
        ref = F.linear(self.qdq(x, x.abs().max()), self.qdq(w, w.abs().amax(dim=1, keepdim=True)))
        assert torch.equal(ref, m(x))

    def test_fake_quant_per_channel_other_precs(self, tq_mod):
        from modelopt_amd.torch.quantization.nn.modules import quant_linear

        di, dw = tq_mod.QAC(num_bits=4), tq_mod.QAC(num_bits=3)
        m = quant_linear.QuantLinear(3, 5, bias=False, quant_desc_input=di, quant_desc_weight=dw).cuda()
        wq, iq = tq_mod.TensorQuantizer(dw), tq_mod.TensorQuantizer(di)
        x = torch.randn(2, 3).cuda()
        assert torch.equal(F.linear(iq(x), wq(m.weight.clone())), m(x))
        ref = F.linear(self.qdq(x, x.abs().max(), 4), self.qdq(m.weight, m.weight.abs().max(), 3))
        assert torch.equal(ref, m(x))

    def test_fake_quant_against_unquantized(self, tq_mod):
        from modelopt_amd.torch.quantization.nn.modules import quant_linear

        x = torch.randn(2, 3).cuda()
        ql = quant_linear.QuantLinear(
            3, 5, bias=True, quant_desc_input=tq_mod.QAC(num_bits=16),
            quant_desc_weight=tq_mod.QAC(num_bits=16, axis=0),
        ).cuda()
        lin = nn.Linear(3, 5, bias=True).cuda()
        lin.load_state_dict(ql.state_dict(), strict=False)
        ql.input_quantizer.disable()
        ql.weight_quantizer.disable()
        assert torch.allclose(ql(x), lin(x))

    def test_set_default_quant_desc(self, tq_mod):
        from modelopt_amd.torch.quantization.nn.modules import quant_linear

        ql = quant_linear.QuantLinear(4, 16)
        assert ql.input_quantizer.axis is None
        assert ql.weight_quantizer.axis == (0)
        try:
            quant_linear.Linear.default_quant_desc_input = tq_mod.QAC(num_bits=11)
            quant_linear.Linear.default_quant_desc_weight = tq_mod.QAC(num_bits=13, axis=1)
            ql = quant_linear.QuantLinear(4, 16)
            assert ql.input_quantizer.num_bits == 11
            assert ql.weight_quantizer.axis == 1
        finally:
            quant_linear.Linear.default_quant_desc_input = tq_mod.tensor_quant.QUANT_DESC_8BIT_PER_TENSOR
            quant_linear.Linear.default_quant_desc_weight = tq_mod.tensor_quant.QUANT_DESC_8BIT_LINEAR_WEIGHT_PER_ROW


# ------------------------------------------------------------------------------------------------
# unit/torch/quantization/test_custom_backend.py:33-110 (register_quant_backend, quantizer cache)
# ------------------------------------------------------------------------------------------------
def _backend_cfg(cfg):
    return {
        "quant_cfg": [
            {"quantizer_name": "*", "enable": False},
            {"quantizer_name": "*weight_quantizer", "cfg": cfg, "enable": True},
        ],
        "algorithm": "max",
    }


def test_custom_backend_via_quantize(mtq):
    from modelopt_amd.torch.quantization.nn import register_quant_backend, unregister_quant_backend

    def dummy_backend(inputs, tq):
        extra = getattr(tq, "backend_extra_args", None) or {}
        return inputs + extra.get("offset", 1.0)

    register_quant_backend("dummy_backend", dummy_backend)
    try:
        model = nn.Linear(16, 16, bias=False).cuda()
        cfg = _backend_cfg({"num_bits": 8, "axis": None, "backend": "dummy_backend",
                            "backend_extra_args": {"offset": 2.5}})
        inputs = torch.randn(1, 16).cuda()
        mtq.quantize(model, cfg, forward_loop=lambda m: m(inputs))
        assert torch.allclose(model(inputs), inputs @ (model.weight.T + 2.5))
    finally:
        unregister_quant_backend("dummy_backend")


def test_custom_backend_with_quantizer_cache(mtq):
    from modelopt_amd.torch.quantization.nn import (
        TensorQuantizerCache,
        register_quant_backend,
        unregister_quant_backend,
    )

    class DummyCache(TensorQuantizerCache):
        def __init__(self):
            super().__init__()
            self.value = 3.0

    def cached_backend(inputs, tq):
        if tq._quantizer_cache is None:
            tq._quantizer_cache = DummyCache()
        return inputs + tq._quantizer_cache.value

    register_quant_backend("cached_backend", cached_backend)
    try:
        model = nn.Linear(16, 16, bias=False).cuda()
        inputs = torch.randn(1, 16).cuda()
        mtq.quantize(model, _backend_cfg({"backend": "cached_backend"}), forward_loop=lambda m: m(inputs))
        assert model.weight_quantizer._quantizer_cache is None
        model(inputs)
        assert isinstance(model.weight_quantizer._quantizer_cache, DummyCache)
        state = model.weight_quantizer.get_modelopt_state()
        assert not any("_quantizer_cache" in k for k in state)
    finally:
        unregister_quant_backend("cached_backend")


# ------------------------------------------------------------------------------------------------
# unit/torch/quantization/test_utils.py:62-79 (reduce_amax upcasts FP8 inputs)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("fp8_dtype", [torch.float8_e4m3fn, torch.float8_e5m2])
@pytest.mark.parametrize("axis", [None, 0, 1, (0, 1)])
def test_reduce_amax_fp8(gpu, fp8_dtype, axis):
    from modelopt_amd.torch.quantization.utils import core_utils as quant_utils

    ref = torch.tensor([[1.0, -3.0, 2.0], [0.5, -0.25, 4.0]]).cuda()
    out = quant_utils.reduce_amax(ref.to(fp8_dtype), axis=axis)
    expected = quant_utils.reduce_amax(ref, axis=axis)
    assert out.dtype == torch.get_default_dtype()
    assert torch.equal(out, expected)
    assert torch.equal(out.cpu(), R.reduce_amax(ref.cpu(), axis=axis))


# ------------------------------------------------------------------------------------------------
# gpu/torch/quantization/test_quantize_cuda.py:80-163 (test_quantize / test_save_restore) with
# the reference's SimpleLinear (_test_utils/torch/quantization/models.py:44-72) and its
# quantize_model_and_forward / save_restore_test helpers (quantize_common.py:64-112).  Configs the
# build does not implement (SmoothQuant, SVDQuant, local-Hessian, rotation, conv models) are not
# listed; see DESIGN.md §8.
# ------------------------------------------------------------------------------------------------
class SimpleLinear(nn.Module):
    def __init__(self, bias=True, dtype=torch.float32):
        super().__init__()
        self.net = nn.Sequential(
            nn.Linear(16, 32, bias=bias, dtype=dtype), nn.ReLU(),
            nn.Linear(32, 64, bias=bias, dtype=dtype), nn.ReLU(),
            nn.Linear(64, 16, bias=bias, dtype=dtype),
        )

    def forward(self, x):
        return self.net(x)

    @classmethod
    def get_input(cls):
        return torch.randn(2, 16)


def _nvfp4_mse_cfgs():
    act_mse = {
        "quant_cfg": [
            {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": (2, 1), "axis": None,
             "block_sizes": {-1: 16, "type": "static", "scale_bits": (4, 3)}}, "enable": True},
            {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": (2, 1), "axis": None,
             "block_sizes": {-1: 16, "type": "dynamic", "scale_bits": (4, 3)}}, "enable": True},
        ],
        "algorithm": {"method": "mse", "step_size": 0.25, "start_multiplier": 0.25, "stop_multiplier": 2.0},
    }
    sweep = {
        "quant_cfg": [
            {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": (2, 1), "axis": None,
             "block_sizes": {-1: 16, "type": "static", "scale_bits": (4, 3)}}, "enable": True},
            {"quantizer_name": "*input_quantizer", "enable": False},
        ],
        "algorithm": {"method": "mse", "fp8_scale_sweep": True},
    }
    return act_mse, sweep


def _configs():
    import copy

    import modelopt_amd.torch.quantization as m

    awq_full = copy.deepcopy(m.INT4_AWQ_CFG)
    awq_full["algorithm"] = "awq_full"
    awq_clip = copy.deepcopy(m.INT4_AWQ_CFG)
    awq_clip["algorithm"] = "awq_clip"
    fp8_2d = copy.deepcopy(m.FP8_2D_BLOCKWISE_WEIGHT_ONLY_CFG)
    for e in fp8_2d["quant_cfg"]:
        if e.get("quantizer_name") == "*weight_quantizer":
            e.setdefault("cfg", {})["block_sizes"] = {-1: 8, -2: 8}
    act_mse, sweep = _nvfp4_mse_cfgs()
    return {
        "INT8_DEFAULT_CFG": m.INT8_DEFAULT_CFG, "FP8_DEFAULT_CFG": m.FP8_DEFAULT_CFG,
        "W4A8_AWQ_BETA_CFG": m.W4A8_AWQ_BETA_CFG, "INT4_BLOCKWISE_WEIGHT_ONLY_CFG": m.INT4_BLOCKWISE_WEIGHT_ONLY_CFG,
        "INT4_AWQ_CFG": m.INT4_AWQ_CFG, "INT4_AWQ_CLIP_CFG": awq_clip, "INT4_AWQ_FULL_CFG": awq_full,
        "NVFP4_DEFAULT_CFG": m.NVFP4_DEFAULT_CFG, "NVFP4_AWQ_LITE_CFG": m.NVFP4_AWQ_LITE_CFG,
        "NVFP4_AWQ_CLIP_CFG": m.NVFP4_AWQ_CLIP_CFG, "NVFP4_AWQ_FULL_CFG": m.NVFP4_AWQ_FULL_CFG,
        "MXFP8_DEFAULT_CFG": m.MXFP8_DEFAULT_CFG, "MXFP6_DEFAULT_CFG": m.MXFP6_DEFAULT_CFG,
        "MXFP4_DEFAULT_CFG": m.MXFP4_DEFAULT_CFG, "MXINT8_DEFAULT_CFG": m.MXINT8_DEFAULT_CFG,
        "FP8_2D_BLOCKWISE_WEIGHT_ONLY_CFG": fp8_2d, "NVFP4_WEIGHT_ACT_MSE_CFG": act_mse,
        "NVFP4_WEIGHT_MSE_FP8_SWEEP_CFG": sweep,
    }


CONFIG_NAMES = [
    "INT8_DEFAULT_CFG", "FP8_DEFAULT_CFG", "W4A8_AWQ_BETA_CFG", "INT4_BLOCKWISE_WEIGHT_ONLY_CFG",
    "INT4_AWQ_CFG", "INT4_AWQ_CLIP_CFG", "INT4_AWQ_FULL_CFG", "NVFP4_DEFAULT_CFG", "NVFP4_AWQ_LITE_CFG",
    "NVFP4_AWQ_CLIP_CFG", "NVFP4_AWQ_FULL_CFG", "MXFP8_DEFAULT_CFG", "MXFP6_DEFAULT_CFG",
    "MXFP4_DEFAULT_CFG", "MXINT8_DEFAULT_CFG", "FP8_2D_BLOCKWISE_WEIGHT_ONLY_CFG",
    "NVFP4_WEIGHT_ACT_MSE_CFG", "NVFP4_WEIGHT_MSE_FP8_SWEEP_CFG",
]


def _quantize_model_and_forward(mtq, model, config, calib_data):
    from modelopt_amd.torch.quantization.utils.names import is_quantized_linear

    def forward_loop(m, run_backward=False):
        for batch in calib_data:
            out = m(batch)
            if run_backward:
                out.sum().backward()

    model = mtq.quantize(model, config, forward_loop=forward_loop)
    for module in model.modules():
        assert not isinstance(module, nn.Linear) or is_quantized_linear(module)
    model.train()
    forward_loop(model, run_backward=True)  # forward and STE backward on the quantized model
    return model


@pytest.mark.parametrize("config_name", CONFIG_NAMES)
def test_quantize(mtq, config_name):
    model = SimpleLinear().cuda()
    calib = [model.get_input().cuda() for _ in range(8)]
    _quantize_model_and_forward(mtq, model, _configs()[config_name], calib)


@pytest.mark.parametrize(
    "config_name",
    ["W4A8_AWQ_BETA_CFG", "INT8_DEFAULT_CFG", "NVFP4_WEIGHT_MSE_FP8_SWEEP_CFG", "NVFP4_WEIGHT_ACT_MSE_CFG"],
)
def test_save_restore(mtq, config_name, tmp_path):
    import modelopt_amd.torch.opt as mto

    model_quant, model_ref = SimpleLinear().cuda(), SimpleLinear().cuda()
    calib = [model_quant.get_input().cuda() for _ in range(2)]
    _quantize_model_and_forward(mtq, model_quant, _configs()[config_name], calib)
    model_quant.eval()
    state = mto.modelopt_state(model_quant)
    mto.restore_from_modelopt_state(model_ref, state)
    model_ref.load_state_dict(model_quant.state_dict())
    model_ref.eval()
    assert torch.equal(model_quant(calib[0]), model_ref(calib[0]))
    for name, mq in model_quant.named_modules():
        if name.endswith("quantizer"):
            assert type(mq) is type(dict(model_ref.named_modules())[name]), name
    # the one-file form: mto.save / mto.restore (weights_only load)
    f = tmp_path / "model.pth"
    mto.save(model_quant, f)
    model_new = mto.restore(SimpleLinear().cuda(), f).eval()
    assert torch.equal(model_quant(calib[0]), model_new(calib[0]))


# ------------------------------------------------------------------------------------------------
# unit/torch/quantization/test_quantize_cpu.py:30-500 (configs, save/restore, set_quantizer_*
# semantics) on the device
# ------------------------------------------------------------------------------------------------
class SimpleLinearCuda(SimpleLinear):
    @classmethod
    def get_input(cls):
        return torch.randn(2, 16, device="cuda")


WINT4INT8_CFG = {
    "quant_cfg": [
        {"quantizer_name": "*weight_quantizer", "cfg": [
            {"num_bits": 4, "block_sizes": {-1: 128, "type": "static"}}, {"num_bits": 8, "axis": 0}],
         "enable": True},
        {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 8, "axis": None}, "enable": True},
    ],
    "algorithm": "awq_lite",
}
INT8_MSE_CFG = {
    "quant_cfg": [
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 8, "axis": 0}},
        {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 8, "axis": None}},
    ],
    "algorithm": "mse",
}
STATIC_WEIGHT_DYNAMIC_ACTIVATION_CFG = {
    "quant_cfg": [
        {"quantizer_name": "*", "enable": False},
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 8, "axis": 0}},
        {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 8, "axis": (0, 1), "type": "dynamic"}},
    ],
    "algorithm": "max",
}


@pytest.mark.parametrize(
    "config_name", ["INT8_DEFAULT_CFG", "INT4_BLOCKWISE_WEIGHT_ONLY_CFG", "INT4_AWQ_CFG", "INT4_AWQ_CLIP_CFG",
                    "INT4_AWQ_FULL_CFG", "WINT4INT8_CFG", "INT8_MSE_CFG"],
)
def test_save_restore_unit_configs(mtq, config_name):
    """test_quantize_cpu.py:123-144 (save_restore_test on the unit-test config list)."""
    import modelopt_amd.torch.opt as mto

    cfg = {"WINT4INT8_CFG": WINT4INT8_CFG, "INT8_MSE_CFG": INT8_MSE_CFG}.get(config_name) or _configs()[config_name]
    model_quant, model_ref = SimpleLinearCuda().cuda(), SimpleLinearCuda().cuda()
    calib = [model_quant.get_input() for _ in range(2)]
    _quantize_model_and_forward(mtq, model_quant, cfg, calib)
    model_quant.eval()
    mto.restore_from_modelopt_state(model_ref, mto.modelopt_state(model_quant))
    model_ref.load_state_dict(model_quant.state_dict())
    assert torch.equal(model_quant(calib[0]), model_ref.eval()(calib[0]))


def test_quantize_invalid_cfg(mtq):
    cfg = {"quant_cfg": [{"quantizer_name": "*", "cfg": {"num_bits": 4, "axis": 0, "block_sizes": {-1: 128}}}],
           "algorithm": "max"}
    with pytest.raises(ValidationError, match=r"axis must be None when block_sizes is not None."):
        mtq.quantize(SimpleLinearCuda().cuda(), cfg)


def test_inplace_backward_compatibility(mtq):
    model = SimpleLinearCuda().cuda()
    calib = [model.get_input() for _ in range(2)]

    def forward_loop():
        for b in calib:
            model(b)

    with pytest.warns(DeprecationWarning):
        mtq.quantize(model, mtq.INT8_DEFAULT_CFG, forward_loop=forward_loop)


def test_custom_calib_config(mtq):
    import modelopt_amd.torch.opt as mto
    from modelopt_amd.torch.quantization.calib import MaxCalibrator

    class NewMaxCalibrator(MaxCalibrator):
        def compute_amax(self):
            return 2 * self._calib_amax

    cfg = {"quant_cfg": [{"quantizer_name": "*", "cfg": {"num_bits": 4, "axis": None,
           "calibrator": (NewMaxCalibrator, (4, None, False))}, "enable": True}], "algorithm": "max"}
    model_ref = mtq.quantize(SimpleLinearCuda().cuda(), cfg, lambda m: m(m.get_input()))
    model_quant = mto.restore_from_modelopt_state(SimpleLinearCuda().cuda(), mto.modelopt_state(model_ref))
    model_quant.load_state_dict(model_ref.state_dict())
    x = model_ref.get_input()
    assert torch.equal(model_ref(x), model_quant(x))
    for name, module in model_quant.named_modules():
        if name.endswith("quantizer"):
            assert module._calibrator.__class__ == NewMaxCalibrator


def test_static_weight_dynamic_activations(mtq):
    model = mtq.quantize(SimpleLinearCuda().cuda(), STATIC_WEIGHT_DYNAMIC_ACTIVATION_CFG, lambda m: m(m.get_input()))
    for name, module in model.named_modules():
        if name.endswith("weight_quantizer"):
            assert module.amax is not None
    model(SimpleLinearCuda.get_input())
    model = mtq.quantize(SimpleLinearCuda().cuda(), STATIC_WEIGHT_DYNAMIC_ACTIVATION_CFG)
    for name, module in model.named_modules():
        if name.endswith("weight_quantizer"):
            assert module.amax is not None


def test_block_sizes_axis_model(mtq):
    import copy

    ref_cfg = {"quant_cfg": [
        {"quantizer_name": "*", "enable": False},
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 8, "axis": 0}},
        {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 8, "axis": None, "type": "dynamic"}},
    ], "algorithm": "max"}
    cfg = {"quant_cfg": [
        {"quantizer_name": "*", "enable": False},
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 8, "block_sizes": {1: None}}},
        {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 8, "block_sizes": {0: None, 1: None}, "type": "dynamic"}},
    ], "algorithm": "max"}
    model_ref = SimpleLinearCuda().cuda()
    model = copy.deepcopy(model_ref)
    x = model_ref.get_input()
    mtq.quantize(model_ref, ref_cfg, lambda m: m(x))
    mtq.quantize(model, cfg, lambda m: m(x))
    assert torch.equal(model_ref(x), model(x))
    for (nr, mr), (n, m) in zip(model_ref.named_modules(), model.named_modules()):
        if hasattr(mr, "weight_quantizer"):
            assert nr == n and torch.equal(mr.weight_quantizer.amax, m.weight_quantizer.amax)


def test_quantize_twice(mtq):
    model = SimpleLinearCuda().cuda()
    x = model.get_input()
    model = mtq.quantize(model, mtq.INT8_DEFAULT_CFG, lambda m: m(x))
    out1 = model(x)
    model = mtq.quantize(model, mtq.INT8_DEFAULT_CFG, lambda m: m(x))
    assert torch.equal(out1, model(x))


class TestSetQuantizerAttributesFull:
    @staticmethod
    def _quantize(mtq, model):
        return mtq.quantize(model, mtq.INT8_DEFAULT_CFG, lambda m: m(m.get_input()))

    def test_basic_full_replacement(self, mtq, tq_mod):
        from modelopt_amd.torch.quantization.conversion import set_quantizer_attributes_full

        model = self._quantize(mtq, SimpleLinearCuda().cuda())
        set_quantizer_attributes_full(model, "*weight_quantizer", tq_mod.QAC(num_bits=4, axis=0))
        for name, module in model.named_modules():
            if name.endswith("weight_quantizer"):
                assert isinstance(module, tq_mod.TensorQuantizer) and module.num_bits == 4 and module.axis == 0

    def test_atomicity_unset_fields_revert_to_defaults(self, mtq, tq_mod):
        from modelopt_amd.torch.quantization.conversion import set_quantizer_attributes_full

        model = self._quantize(mtq, SimpleLinearCuda().cuda())
        set_quantizer_attributes_full(model, "*weight_quantizer", tq_mod.QAC(num_bits=8, axis=0))
        set_quantizer_attributes_full(model, "*weight_quantizer", tq_mod.QAC(num_bits=4))
        for name, module in model.named_modules():
            if name.endswith("weight_quantizer"):
                assert module.num_bits == 4 and module.axis == tq_mod.QAC().axis

    def test_wildcard_no_match_is_noop(self, mtq, tq_mod):
        from modelopt_amd.torch.quantization.conversion import set_quantizer_attributes_full

        model = self._quantize(mtq, SimpleLinearCuda().cuda())
        before = {n: m.num_bits for n, m in model.named_modules() if isinstance(m, tq_mod.TensorQuantizer)}
        set_quantizer_attributes_full(model, "*nonexistent_quantizer*", tq_mod.QAC(num_bits=4))
        assert before == {n: m.num_bits for n, m in model.named_modules() if isinstance(m, tq_mod.TensorQuantizer)}

    def test_invalid_attributes_type_raises(self, mtq):
        from modelopt_amd.torch.quantization.conversion import set_quantizer_attributes_full

        model = self._quantize(mtq, SimpleLinearCuda().cuda())
        with pytest.raises((ValueError, AttributeError)):
            set_quantizer_attributes_full(model, "*weight_quantizer", {"num_bits": 4})

    def test_list_attributes_creates_sequential_quantizer(self, mtq, tq_mod):
        from modelopt_amd.torch.quantization.conversion import set_quantizer_attributes_full

        model = self._quantize(mtq, SimpleLinearCuda().cuda())
        attrs = [tq_mod.QAC(num_bits=4, block_sizes={-1: 128}), tq_mod.QAC(num_bits=8, axis=0)]
        set_quantizer_attributes_full(model, "*weight_quantizer", attrs)
        for name, module in model.named_modules():
            if name.endswith("weight_quantizer"):
                assert isinstance(module, tq_mod.SequentialQuantizer) and len(module) == 2


def test_ordering_later_entry_overrides_earlier(mtq):
    cfg = {"quant_cfg": [
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 8, "axis": 0}},
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4, "axis": 0}},
        {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 8, "axis": None}},
    ], "algorithm": "max"}
    model = mtq.quantize(SimpleLinearCuda().cuda(), cfg, lambda m: m(m.get_input()))
    for name, module in model.named_modules():
        if name.endswith("weight_quantizer"):
            assert module.num_bits == 4
        if name.endswith("input_quantizer"):
            assert module.num_bits == 8


def test_enable_only_entry_preserves_attributes(mtq):
    cfg = {"quant_cfg": [
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4, "axis": 0}},
        {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 8, "axis": None}},
        {"quantizer_name": "*weight_quantizer", "enable": False},
    ], "algorithm": "max"}
    model = mtq.quantize(SimpleLinearCuda().cuda(), cfg, lambda m: m(m.get_input()))
    for name, module in model.named_modules():
        if name.endswith("weight_quantizer"):
            assert not module.is_enabled and module.num_bits == 4 and module.axis == 0


def test_atomicity_later_cfg_entry_does_not_inherit_earlier(mtq, tq_mod):
    cfg = {"quant_cfg": [
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 8, "axis": 0}},
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4}},
        {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 8, "axis": None}},
    ], "algorithm": "max"}
    model = mtq.quantize(SimpleLinearCuda().cuda(), cfg, lambda m: m(m.get_input()))
    for name, module in model.named_modules():
        if name.endswith("weight_quantizer"):
            assert module.num_bits == 4 and module.axis == tq_mod.QAC().axis


def test_legacy_dict_format_end_to_end(mtq, tq_mod):
    old = {"quant_cfg": {"default": {"enable": False}, "*weight_quantizer": {"num_bits": 8, "axis": 0},
                         "*input_quantizer": {"num_bits": 8, "axis": None}}, "algorithm": "max"}
    model = mtq.quantize(SimpleLinearCuda().cuda(), old, lambda m: m(m.get_input()))
    for name, module in model.named_modules():
        if isinstance(module, tq_mod.TensorQuantizer):
            if name.endswith(("weight_quantizer", "input_quantizer")):
                assert module.is_enabled and module.num_bits == 8
            elif name.endswith("output_quantizer"):
                assert not module.is_enabled


# ------------------------------------------------------------------------------------------------
# unit/torch/quantization/test_calibrator.py:28-354 (Max / Histogram / Entropy / MSE / Percentile
# calibrators) on device tensors; amax values also checked against the oracle's calibrators
# (oracle/ref_ops.py, the reference's histogram.py restated on the CPU).
# ------------------------------------------------------------------------------------------------
def _calib(gpu):
    from modelopt_amd.torch.quantization import calib

    return calib


class TestMaxCalibrator:
    def test_simple_run(self, gpu):
        c = _calib(gpu).MaxCalibrator(8, None, False)
        x1, x2 = torch.rand(16).cuda(), torch.rand(16).cuda()
        c.collect(x1)
        c.collect(x2)
        assert torch.equal(c.compute_amax(), torch.max(x1.max(), x2.max()))
        _calib(gpu).MaxCalibrator(8, None, True)

    @pytest.mark.parametrize("axis", [0, -4])
    def test_fine_grain(self, gpu, axis):
        from modelopt_amd.torch.quantization.utils import core_utils as quant_utils

        c = _calib(gpu).MaxCalibrator(8, axis, False)
        x1, x2 = torch.rand(3, 4, 2, 2).cuda(), torch.rand(3, 4, 2, 2).cuda()
        c.collect(x1)
        c.collect(x2)
        assert c.compute_amax().shape[0] == 3
        assert torch.equal(c.compute_amax(), quant_utils.reduce_amax(torch.max(x1, x2), axis=(1, 2, 3)))
        c.reset()
        assert c.compute_amax() is None

    def test_track_amax(self, gpu):
        import numpy as np

        c = _calib(gpu).MaxCalibrator(8, None, False, track_amax=True)
        x1, x2 = torch.rand(16).cuda(), torch.rand(16).cuda()
        c.collect(x1)
        c.collect(x2)
        assert torch.equal(c.compute_amax(), torch.max(x1.max(), x2.max()))
        np.testing.assert_array_equal(c.amaxs[0], x1.max().cpu().numpy())
        np.testing.assert_array_equal(c.amaxs[1], x2.max().cpu().numpy())

    def test_track_amax_raises(self, gpu):
        c = _calib(gpu).MaxCalibrator(8, 0, False)
        c.collect(torch.rand(3, 4, 2, 2).cuda())
        with pytest.raises(RuntimeError, match="shape changed"):
            c.collect(torch.rand(4, 4, 2, 2).cuda())


def _hist_pair(gpu, *args, **kwargs):
    """(device calibrator, oracle calibrator) with the same arguments."""
    num_bits, _axis, unsigned = args
    dev = _calib(gpu).HistogramCalibrator(num_bits, None, unsigned, **kwargs)
    kw = {k: v for k, v in kwargs.items() if k in ("num_bins", "skip_zeros")}
    ref = R.HistogramCalibratorRef(num_bits, unsigned, **kw)
    return dev, ref


class TestHistogramCalibrator:
    def test_skip_zeros(self, gpu):
        dev, ref = _hist_pair(gpu, 8, None, False, num_bins=2048, skip_zeros=True)
        for x in (torch.tensor([0, 0, 0, 0, 0, 1, 2, 3, 4, 5]), torch.tensor([0, 0, 0, 0, 0, 6, 7, 8, 9, 10])):
            dev.collect(x.cuda())
            ref.collect(x)
        amax = dev.compute_amax("percentile", percentile=50, start_bin=128)
        assert (amax - 5.0).abs() < 10 / 2048
        assert float(amax) == float(ref.compute_amax("percentile", percentile=50, start_bin=128))

    def test_torch_hist_growth(self, gpu):
        """test_torch_hist (test_calibrator.py:141-181): histogram / edges through range growth,
        here against the oracle's torch-branch restatement (the numpy branch is not built)."""
        torch.manual_seed(0)
        x1 = torch.rand(15)
        x1[0] = 0
        x2 = torch.rand(15) + 1
        x2[1] = 0
        dev, ref = _hist_pair(gpu, 8, None, False, num_bins=19)
        for x in [x1] + [x2, x1] * 3:
            dev.collect(x.cuda())
            ref.collect(x)
            assert dev._calib_hist.numel() == dev._calib_bin_edges.numel() - 1
            assert torch.equal(dev._calib_hist.cpu(), ref._calib_hist.cpu())
            assert torch.allclose(dev._calib_bin_edges.cpu().double(), ref._calib_bin_edges.cpu().double())
        dev.compute_amax("percentile", percentile=99.99)


class TestEntropyCalibrator:
    @pytest.mark.parametrize("unsigned", [False, True])
    def test_one_tensor(self, gpu, unsigned):
        dev, ref = _hist_pair(gpu, 8, None, unsigned, num_bins=512, grow_method="stretch")
        x = torch.rand(11, 7, 3, 3)
        x[1, 1, 1, 1] = 10.0
        dev.collect(x.cuda())
        ref.collect(x)
        amax = dev.compute_amax("entropy", start_bin=32)
        assert amax < 1.1
        assert float(amax) == float(ref.compute_amax("entropy", start_bin=32))

    def test_two_tensor(self, gpu):
        dev = _calib(gpu).HistogramCalibrator(8, None, False, num_bins=512)
        x2 = torch.rand(11, 7, 3, 3)
        x2[1, 1, 1, 1] = 10.0
        dev.collect(x2.cuda())
        dev.collect(torch.rand(11, 7, 3, 3).cuda())
        assert dev.compute_amax("entropy", start_bin=32) < 1.1

    def test_repr(self, gpu):
        repr(_calib(gpu).HistogramCalibrator(8, None, True, num_bins=2048))


class TestMSECalibrator:
    def test_one_tensor(self, gpu):
        c = _calib(gpu).HistogramCalibrator(8, None, False, num_bins=32)
        x = torch.ones(4, 4, 4) * 255.0
        x[1, 1, 1] = 256.0
        c.collect(x.cuda())
        amax = c.compute_amax("mse", start_bin=16)
        assert (amax - 255.0).abs() < (amax - 256.0).abs()

    def test_unsigned_one_tensor(self, gpu):
        c = _calib(gpu).HistogramCalibrator(8, None, True, num_bins=32)
        x = torch.ones(11, 7, 3, 3) * 512.0
        x[1, 1, 1, 1] = 513.0
        c.collect(x.cuda())
        amax = c.compute_amax("mse", start_bin=8)
        assert (amax - 512.0).abs() < (amax - 513.0).abs()

    def test_two_tensor(self, gpu):
        c = _calib(gpu).HistogramCalibrator(8, None, False)
        x1 = torch.ones(11, 7, 3, 3) * 255.0
        x1[1, 1, 1, 1] = 256.0
        c.collect(x1.cuda())
        c.collect((torch.ones(11, 7, 3, 3) * 255.0).cuda())
        amax = c.compute_amax("mse")
        assert (amax - 255.0).abs() < (amax - 256.0).abs()


class TestPercentileCalibrator:
    @pytest.mark.parametrize(("unsigned", "pct", "want", "tol"), [(False, 90, 89.0, 100 / 1024), (True, 80, 79.0, 100 / 2048)])
    def test_one_tensor(self, gpu, unsigned, pct, want, tol):
        dev, ref = _hist_pair(gpu, 8, None, unsigned)
        x = torch.arange(100)
        dev.collect(x.cuda())
        ref.collect(x.float())
        amax = dev.compute_amax("percentile", percentile=pct)
        assert (amax - want).abs() < tol
        assert float(amax) == float(ref.compute_amax("percentile", percentile=pct))

    def test_two_tensor(self, gpu):
        c = _calib(gpu).HistogramCalibrator(8, None, False)
        c.collect(torch.arange(100).cuda())
        c.collect(torch.arange(0, 50, 0.5).cuda())
        amax = c.compute_amax("percentile", percentile=99)
        assert (amax - 97.0).abs() < 100 / 1024

    def test_range(self, gpu):
        c = _calib(gpu).HistogramCalibrator(8, None, False)
        c.collect(torch.arange(100).cuda())
        with pytest.raises(ValueError, match="range"):
            c.compute_amax("percentile", percentile=-10)
        with pytest.raises(ValueError, match="range"):
            c.compute_amax("percentile", percentile=200)
