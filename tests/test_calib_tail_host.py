"""The calibration tail on the host path: finish_stats_collection's adopted amax equals the
reference-shaped load_calib_amax result (value, dtype, shape) and does not alias the calibrator's
running buffer; the batched validation flags negative / NaN / inf amax as validate_attr does
(reference tensor_quantizer.py:693-720, :757-773; model_quant.py:121-127)."""
import warnings

import torch
from torch import nn

from modelopt_amd.torch.quantization import model_calib as MC
from modelopt_amd.torch.quantization.calib.max import _bad_flags
from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig
from modelopt_amd.torch.quantization.model_quant import _validate_quantizer_attrs
from modelopt_amd.torch.quantization.nn.modules.tensor_quantizer import TensorQuantizer


def _calibrated(dtype, axis):
    q = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, axis=axis))
    q.disable_quant()
    q.enable_calib()
    g = torch.Generator().manual_seed(3)
    for _ in range(3):
        q(torch.randn(16, 32, generator=g).to(dtype))
    return q


def test_finish_adopts_same_amax_as_load_calib_amax():
    for dtype in (torch.float32, torch.bfloat16):
        for axis in (None, 0):
            ref, got = _calibrated(dtype, axis), _calibrated(dtype, axis)
            ref.load_calib_amax()
            holder = nn.Module()
            holder.q = got
            MC.finish_stats_collection(holder)
            assert got.amax.dtype == ref.amax.dtype and got.amax.shape == ref.amax.shape
            assert torch.equal(got.amax, ref.amax), (dtype, axis)
            got._calibrator._acc.fill_(1e9)  # the adopted buffer is not the running max
            assert torch.equal(got.amax, ref.amax)
            assert got._if_quant and not got._if_calib


def test_bad_flags_host():
    x = torch.tensor([0.5, 1.0, 2.0])
    assert _bad_flags(x).tolist() == [0, 0, 0]
    assert _bad_flags(torch.tensor([float("nan"), 1.0])).tolist() == [1, 0, 0]
    assert _bad_flags(torch.tensor([float("inf"), 1.0])).tolist() == [0, 1, 0]
    assert _bad_flags(torch.tensor([-1.0, 1.0])).tolist() == [0, 0, 1]


def test_validate_attrs_warns_on_negative_amax():
    holder = nn.Module()
    holder.q = TensorQuantizer(QuantizerAttributeConfig(num_bits=8))
    holder.q.amax = torch.tensor(-1.0)
    holder.ok = TensorQuantizer(QuantizerAttributeConfig(num_bits=8))
    holder.ok.amax = torch.tensor(2.0)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        _validate_quantizer_attrs(holder)
    assert any("q" in str(m.message) for m in w)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        _validate_quantizer_attrs(nn.ModuleDict({"ok": holder.ok}))
    assert not w


def test_static_block_quantizer_recalibrated_keeps_fp32_amax():
    """A promoted StaticBlockScaleQuantizer max-calibrated again after reset_amax keeps its amax
    in fp32 (its _amax_setter_helper override), not in the input dtype."""
    import torch
    import torch.nn as nn

    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.nn.modules.tensor_quantizer import StaticBlockScaleQuantizer

    cfg = {
        "quant_cfg": [
            {"quantizer_name": "*", "enable": False},
            {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4, "block_sizes": {-1: 8, "type": "static"}}},
        ],
        "algorithm": "max",
    }
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(16, 16)).to(torch.bfloat16)
    mtq.quantize(m, cfg, lambda mm: mm(torch.randn(4, 16, dtype=torch.bfloat16)))
    q = m[0].weight_quantizer
    assert isinstance(q, StaticBlockScaleQuantizer) and q._amax.dtype == torch.float32
    q.reset_amax()
    mtq.calibrate(m, "max", lambda mm: mm(torch.randn(4, 16, dtype=torch.bfloat16)))
    assert q._amax.dtype == torch.float32
    want = m[0].weight.detach().float().view(-1, 8).abs().amax(dim=1, keepdim=True)
    assert torch.equal(q._amax.view(-1, 1), want)
