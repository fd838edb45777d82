"""HIP path vs the reference's own outputs (golden fixtures made by running the reference).

Bit-exact for every fake-quant and amax case (INT, FP8, block, padding, calibrators, histogram
including the entropy/percentile amax); MX against the reference's known-answer tables.
"""

import json
from pathlib import Path

import pytest
import torch
from safetensors.torch import load_file

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"


def same_bits(a, b):
    a, b = a.detach().cpu(), b.detach().cpu()
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    nan = torch.isnan(a.float()) & torch.isnan(b.float())
    iv = {torch.float32: torch.int32, torch.float16: torch.int16, torch.bfloat16: torch.int16}[a.dtype]
    return bool(((a.view(iv) == b.view(iv)) | nan).all())


@pytest.fixture(scope="module")
def tq():
    return load_file(str(G / "tensor_quant.safetensors")), json.loads((G / "tensor_quant.json").read_text())


def test_functional_cases(gpu, tq):
    from modelopt_amd.torch.quantization import tensor_quant as T

    t, meta = tq
    for m in meta:
        x = t[m["x"]].to(gpu)
        amax = t[m["amax"]].to(gpu)
        if m.get("fp8"):
            y = T.scaled_e4m3(x * m["x_scale"], amax, None, 4, 3)
        else:
            xi = x.abs() if m["abs"] else x
            y = T.fake_tensor_quant(xi, amax, None, m["num_bits"], m["unsigned"], m["narrow_range"])
        assert same_bits(y, t[m["key"] + "_y"]), m["key"]


@pytest.mark.parametrize("dn", ["f32", "f16", "bf16"])
def test_block_cast_amax(gpu, tq, dn):
    from modelopt_amd.torch.quantization import tensor_quant as T
    from modelopt_amd.torch.quantization.utils import reduce_amax

    t, _ = tq
    x, a = t[f"blk_{dn}_x"].to(gpu), t[f"blk_{dn}_amax"].to(gpu)
    assert same_bits(T.fp8_fake_quant(x, a), t[f"fp8blk_{dn}_y"])
    assert same_bits(T.fake_tensor_quant(x, a, None, 4, False, False), t[f"int4blk_{dn}_y"])
    assert same_bits(T.e4m3_cast(t[f"fp8cast_{dn}_x"].to(gpu)), t[f"fp8cast_{dn}_y"])
    xr = t[f"amax_{dn}_x"].to(gpu)
    for name, ax in [("all", None), ("a0", [0]), ("a2", [2]), ("a01", [0, 1]), ("a02", [0, 2]), ("a12", [1, 2])]:
        assert same_bits(reduce_amax(xr, axis=ax), t[f"amax_{dn}_{name}"]), name


def test_fp8_special_values(gpu, tq):
    from modelopt_amd.torch.quantization import tensor_quant as T

    t, _ = tq
    for a in [448.0, 3.0, 0.0, 1e-30]:
        y = T.fp8_fake_quant(t["fp8sv_x"].to(gpu), torch.tensor(a, device=gpu))
        assert same_bits(y, t[f"fp8sv_{a}_y"]), a


def _calib_then_quant(gpu, cfg, x, y=None):
    from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig
    from modelopt_amd.torch.quantization.nn import TensorQuantizer

    q = TensorQuantizer(QuantizerAttributeConfig(**cfg)).to(gpu)
    q.enable_calib()
    q.disable_quant()
    q(x.to(gpu))
    q.load_calib_amax()
    q.disable_calib()
    q.enable_quant()
    return q, q((x if y is None else y).to(gpu))


@pytest.mark.parametrize("dn", ["f32", "f16", "bf16"])
@pytest.mark.parametrize(
    "case,cfg",
    [
        ("int8_tensor", {"num_bits": 8}),
        ("int8_axis0", {"num_bits": 8, "axis": 0}),
        ("int8_axism1", {"num_bits": 8, "axis": -1}),
        ("fp8_tensor", {"num_bits": (4, 3)}),
        ("int4_b128", {"num_bits": 4, "block_sizes": {-1: 128, "type": "static"}}),
        ("fp8_b128", {"num_bits": (4, 3), "block_sizes": {-1: 128}}),
    ],
)
def test_tensor_quantizer_cases(gpu, dn, case, cfg):
    t = load_file(str(G / "quantizer.safetensors"))
    k = f"q_{dn}_{case}"
    q, out = _calib_then_quant(gpu, cfg, t[k + "_x"], t.get(k + "_y_in"))
    assert same_bits(q.amax, t[k + "_amax"]), "amax"
    assert same_bits(out, t[k + "_out"]), "out"


def test_block_padding_cases(gpu):
    from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig
    from modelopt_amd.torch.quantization.nn import TensorQuantizer

    t = load_file(str(G / "quantizer.safetensors"))
    q, out = _calib_then_quant(gpu, {"num_bits": 8, "block_sizes": {-1: 2}}, t["blk_simple_padding_x"])
    assert same_bits(q.amax, t["blk_simple_padding_amax"]) and same_bits(out, t["blk_simple_padding_out"])
    q, out = _calib_then_quant(gpu, {"num_bits": 8, "block_sizes": {-1: 2, 1: 3}}, t["blk_complex_padding_x"])
    assert same_bits(q.amax, t["blk_complex_padding_amax"]) and same_bits(out, t["blk_complex_padding_out"])
    q = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, block_sizes={-1: 2, 1: 3}))
    assert same_bits(q(t["blk_complex_x"].to(gpu)), t["blk_complex_out"])
    q = TensorQuantizer(QuantizerAttributeConfig(num_bits=(4, 3), type="dynamic", block_sizes={-1: None, "type": "dynamic"}))
    assert same_bits(q(t["fp8_per_token_x"].to(gpu)), t["fp8_per_token_out"])


def test_calibrators(gpu):
    from modelopt_amd.torch.quantization.calib import HistogramCalibrator, MaxCalibrator

    t = load_file(str(G / "calib.safetensors"))
    meta = json.loads((G / "calib.json").read_text())
    xs = [t[f"batch{i}"].to(gpu) for i in range(3)]
    for name, axis in [("none", None), ("a0", 0), ("a1", 1)]:
        c = MaxCalibrator(8, axis, False)
        for x in xs:
            c.collect(x)
        assert same_bits(c.compute_amax(), t[f"max_{name}"]), name
    h = HistogramCalibrator(8, None, False, num_bins=256)
    for x in xs:
        h.collect(x)
    assert torch.equal(h._calib_hist.cpu(), t["hist"])
    assert torch.equal(h._calib_bin_edges.cpu(), t["hist_edges"])
    assert h._num_bins == meta["hist_num_bins"]
    assert float(h.compute_amax("entropy", start_bin=128)) == meta["entropy"]
    assert float(h.compute_amax("percentile", percentile=99.0)) == meta["percentile_99"]
    assert float(h.compute_amax("percentile", percentile=99.99)) == meta["percentile_9999"]
    h2 = HistogramCalibrator(8, None, False, num_bins=2048, skip_zeros=True)
    h2.collect(t["hist_skip_zeros_x"].to(gpu))
    assert torch.equal(h2._calib_hist.cpu(), t["hist_skip_zeros"])


def test_max_calibrator_lazy_nan_assert(gpu):
    from modelopt_amd.torch.quantization.calib import MaxCalibrator

    c = MaxCalibrator()
    x = torch.randn(64, 64, device=gpu)
    x[3, 3] = float("nan")
    c.collect(x)  # no host sync here
    with pytest.raises(AssertionError):
        c.compute_amax()


def _kat_cases():
    kat = json.loads((G / "mx_kat.json").read_text())
    fmt_name = {(2, 1): "E2M1", (3, 2): "E3M2", (2, 3): "E2M3", (4, 3): "E4M3", (5, 2): "E5M2", 8: "INT8"}
    out = []
    for test, d in kat.items():
        for o in d["outputs"]:
            f = tuple(o["format"]) if isinstance(o["format"], list) else o["format"]
            for bs in ([d["block_size"]] if d["block_size"] else [8, 16, 32]):
                for dt in ([torch.float32, torch.float16, torch.bfloat16] if test == "test_mxfp4" else [torch.float32]):
                    out.append((test, fmt_name[f], bs, dt, d["input"], o["expected"]))
    return out


@pytest.mark.parametrize("case", _kat_cases(), ids=lambda c: f"{c[0]}-{c[1]}-bs{c[2]}-{str(c[3])[6:]}")
def test_mx_known_answers(gpu, case):
    from modelopt_amd.torch.quantization.extensions import get_cuda_ext_mx

    ext = get_cuda_ext_mx(raise_if_failed=True)
    _, fmt, bs, dt, inp, exp = case
    x = torch.tensor(inp, dtype=torch.float32)
    y = torch.tensor(exp, dtype=torch.float32)
    rep = max(bs // x.shape[1], 1)
    x, y = x.repeat(1, rep), y.repeat(1, rep)
    sign = (torch.randint(0, 2, x.shape, generator=torch.Generator().manual_seed(0)) * 2 - 1).float()
    xi = (x * sign).to(dt).to(gpu)
    out = ext.fused_amax_convert(xi, bs, getattr(ext.Types, fmt), ext.Types.E8M0, None)
    assert out.dtype == xi.dtype
    # reference tolerance (test_quantize_mxformats_cuda.py) ...
    assert torch.allclose(out.float().cpu(), (y * sign).to(dt).float(), atol=1e-3)
    # ... and bit-exact against the oracle's table walk on the same input
    ref = R.fused_amax_convert(xi.cpu(), bs, fmt)
    assert torch.equal(out.cpu().float(), ref.float())
