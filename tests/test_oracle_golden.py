"""Pin the oracle: oracle/ref_ops.py vs golden vectors produced by the reference itself.

The goldens (tests/golden/*.safetensors, made by tests/golden/make_golden.py from /root/reference)
hold inputs and the reference's outputs; every oracle function must reproduce them exactly (MX:
the reference's own known-answer tables, with its tolerance, plus exactness on the table values).
CPU only.
"""

import json
from pathlib import Path

import pytest
import torch
from safetensors.torch import load_file

from oracle import ref_ops as R

G = Path(__file__).resolve().parent / "golden"


def bits_equal(a, b):
    a, b = a.detach(), b.detach()
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    nan = torch.isnan(a.float()) & torch.isnan(b.float())
    iv = {torch.float32: torch.int32, torch.float16: torch.int16, torch.bfloat16: torch.int16}[a.dtype]
    return bool(((a.view(iv) == b.view(iv)) | nan).all())


@pytest.fixture(scope="module")
def tq():
    return load_file(str(G / "tensor_quant.safetensors")), json.loads((G / "tensor_quant.json").read_text())


def test_int_and_fp8_cases(tq):
    t, meta = tq
    n = 0
    for m in meta:
        x = t[m["x"]]
        amax = t[m["amax"]]
        if m.get("fp8"):
            y = R.fp8_eager(x * m["x_scale"], amax)
        else:
            xi = x.abs() if m["abs"] else x
            y = R.tensor_quant(xi, amax, m["num_bits"], m["unsigned"], m["narrow_range"])
        assert bits_equal(y, t[m["key"] + "_y"]), m["key"]
        n += 1
    assert n == 3 * 3 * 6


@pytest.mark.parametrize("dn", ["f32", "f16", "bf16"])
def test_block_and_cast(tq, dn):
    t, _ = tq
    x, a = t[f"blk_{dn}_x"], t[f"blk_{dn}_amax"]
    assert bits_equal(R.fp8_eager(x, a), t[f"fp8blk_{dn}_y"])
    assert bits_equal(R.tensor_quant(x, a, 4, False, False), t[f"int4blk_{dn}_y"])
    assert bits_equal(R.fp8_eager(t[f"fp8cast_{dn}_x"], None), t[f"fp8cast_{dn}_y"])


@pytest.mark.parametrize("dn", ["f32", "f16", "bf16"])
def test_reduce_amax(tq, dn):
    t, _ = tq
    x = t[f"amax_{dn}_x"]
    for name, ax in [("all", None), ("a0", [0]), ("a2", [2]), ("a01", [0, 1]), ("a02", [0, 2]), ("a12", [1, 2])]:
        assert bits_equal(R.reduce_amax(x, axis=ax), t[f"amax_{dn}_{name}"]), name


def test_fp8_special_values(tq):
    t, _ = tq
    for a in [448.0, 3.0, 0.0, 1e-30]:
        assert bits_equal(R.fp8_eager(t["fp8sv_x"], torch.tensor(a)), t[f"fp8sv_{a}_y"])


def test_calibrators():
    t = load_file(str(G / "calib.safetensors"))
    meta = json.loads((G / "calib.json").read_text())
    xs = [t[f"batch{i}"] for i in range(3)]
    for name, axis in [("none", None), ("a0", 0), ("a1", 1)]:
        c = R.MaxCalibratorRef(axis)
        for x in xs:
            c.collect(x)
        assert bits_equal(c.compute_amax(), t[f"max_{name}"])
    h = R.HistogramCalibratorRef(8, False, num_bins=256)
    for x in xs:
        h.collect(x)
    assert torch.equal(h._calib_hist, t["hist"])
    assert torch.equal(h._calib_bin_edges, t["hist_edges"])
    assert h._num_bins == meta["hist_num_bins"]
    assert float(h.compute_amax("entropy", start_bin=128)) == meta["entropy"]
    assert float(h.compute_amax("percentile", percentile=99.0)) == meta["percentile_99"]
    assert float(h.compute_amax("percentile", percentile=99.99)) == meta["percentile_9999"]
    h2 = R.HistogramCalibratorRef(8, False, num_bins=2048, skip_zeros=True)
    h2.collect(t["hist_skip_zeros_x"])
    assert torch.equal(h2._calib_hist, t["hist_skip_zeros"])


def _kat_cases():
    kat = json.loads((G / "mx_kat.json").read_text())
    fmt_name = {(2, 1): "E2M1", (3, 2): "E3M2", (2, 3): "E2M3", (4, 3): "E4M3", (5, 2): "E5M2", 8: "INT8"}
    cases = []
    for test, d in kat.items():
        for o in d["outputs"]:
            f = tuple(o["format"]) if isinstance(o["format"], list) else o["format"]
            for bs in ([d["block_size"]] if d["block_size"] else [8, 16, 32]):
                cases.append((test, fmt_name[f], bs, d["input"], o["expected"]))
    return cases


@pytest.mark.parametrize("case", _kat_cases(), ids=lambda c: f"{c[0]}-{c[1]}-bs{c[2]}")
def test_mx_oracle_known_answers(case):
    """Reference KATs (test_quantize_mxformats_cuda.py:61-317): inputs repeated to the block size,
    random signs, allclose(atol=1e-3) as in the reference."""
    _, fmt, bs, inp, exp = case
    x = torch.tensor(inp, dtype=torch.float32)
    y = torch.tensor(exp, dtype=torch.float32)
    rep = max(bs // x.shape[1], 1)
    x, y = x.repeat(1, rep), y.repeat(1, rep)
    sign = (torch.randint(0, 2, x.shape, generator=torch.Generator().manual_seed(0)) * 2 - 1).float()
    out = R.fused_amax_convert(x * sign, bs, fmt)
    assert torch.allclose(out, y * sign, atol=1e-3), (out - y * sign).abs().max()


def test_mx_oracle_e2m1_boundaries():
    """E2M1 tie/boundary table (test_tensor_quant_cuda.py:182-268): exact."""
    x = torch.tensor([[0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5.0, 6.0]])
    out = R.convert_to_types(x, "E2M1")
    assert out.tolist() == [[0.0, 1.0, 1.0, 2.0, 2.0, 4.0, 4.0, 6.0]]


def test_nvfp4_oracle_matches_reference_triton_kernel():
    """oracle.nvfp4_fake_quant_block == the reference's Triton fp4_fake_quant_block (run through
    the Triton interpreter by tests/golden/make_golden.py) on every block whose FP8 scale the
    interpreter casts like the hardware (see gen_nvfp4); the excluded blocks are few."""
    from safetensors.torch import load_file

    t = load_file(str(G / "nvfp4.safetensors"))
    meta = json.loads((G / "nvfp4.json").read_text())
    for name, m in meta.items():
        if "blocks" not in m:
            continue
        x, amax, y, ok = t[f"{name}.x"], t[f"{name}.amax"], t[f"{name}.y"], t[f"{name}.block_ok"].bool()
        assert m["excluded"] <= m["blocks"] // 20
        got = R.nvfp4_fake_quant_block(x, amax)
        rows, cols = x.shape
        okc = ok.repeat_interleave(16, dim=1)[:, :cols]
        assert torch.equal(got[okc], y[okc]), name


def test_nvfp4_static_scales_match_reference():
    """oracle.compute_fp4_scales == the reference's compute_fp4_scales (fp4_kernel.py:217-251)."""
    from safetensors.torch import load_file

    t = load_file(str(G / "nvfp4.safetensors"))
    meta = json.loads((G / "nvfp4.json").read_text())
    for name, m in meta.items():
        if not m.get("static_scales"):
            continue
        amax = t[f"{name}.amax"]
        assert torch.equal(R.compute_fp4_scales(amax, amax.amax()), t[f"{name}.scale"])
        assert torch.equal(R.compute_fp4_scales(amax, amax.amax() * 2), t[f"{name}.scale_g2"])
        assert torch.equal(R.compute_fp4_scales(amax, None, True, 256.0), t[f"{name}.scale_46"])


# ---- MSE weight calibration (calib/mse.py) and AWQ-clip (model_calib.py:1725-1940) ----------


@pytest.fixture(scope="module")
def mse_gold():
    return load_file(str(G / "mse.safetensors")), json.loads((G / "mse.json").read_text())


def test_nvfp4_sweep_oracle_matches_reference_triton_kernel(mse_gold):
    t, meta = mse_gold
    assert torch.equal(R.fp8_scale_candidates(), t["sweep.candidates"])
    for name, m in meta["sweep"].items():
        got = R.nvfp4_fp8_scale_sweep(t[f"sweep.{name}.x"], t[f"sweep.{name}.global_amax"], m["block"])
        assert bits_equal(got, t[f"sweep.{name}.best"]), name


def _mse_quant_fn(name, m):
    if m["cfg"]["num_bits"] == [4, 3]:
        return lambda x, a: R.fp8_eager(x, a)
    nb = m["cfg"]["num_bits"]
    return lambda x, a: R.tensor_quant(x, a, nb, False, False)


def test_mse_sweep_oracle_matches_reference(mse_gold):
    t, meta = mse_gold
    for name, m in meta["cal"].items():
        w = t[f"cal.{name}.w"].float()
        if m["block"]:
            w = w.reshape(-1, m["block"])
        axis = tuple(m["axis"]) if isinstance(m["axis"], list) else m["axis"]
        losses, best = R.mse_sweep(w, t[f"cal.{name}.init_amax"], _mse_quant_fn(name, m), axis)
        assert torch.equal(losses.reshape(losses.shape[0], -1), t[f"cal.{name}.losses"]), name
        assert bits_equal(best, t[f"cal.{name}.best"]), name


@pytest.fixture(scope="module")
def clip_gold():
    return load_file(str(G / "awq_clip.safetensors")), json.loads((G / "awq_clip.json").read_text())


def _layer_inputs(t, name, layers, data_keys):
    """The activations each linear sees in the reference forward (pre_quant_scale applied)."""
    acts = {n: [] for n in layers}
    for dk in data_keys:
        x = t[dk]
        for n in layers:
            pqs = t.get(f"{name}.{n}.pqs")
            xin = x * pqs if pqs is not None else x
            acts[n].append(xin)
            x = torch.nn.functional.linear(xin, t[f"{name}.{n}.weight"])
            if n != layers[-1]:
                x = torch.relu(x)
    return acts


def test_awq_clip_oracle_matches_reference(clip_gold):
    t, meta = clip_gold
    for name, m in meta.items():
        layers = list(m["layers"])
        data_keys = sorted(k for k in t if k.startswith(f"{name}.data"))
        acts = _layer_inputs(t, name, layers, data_keys)
        for n in layers:
            shrinks = m["layers"][n]["shrinks"]
            assert shrinks == R.awq_clip_shrinks()
            w, w_amax = t[f"{name}.{n}.weight"], t[f"{name}.{n}.w_amax"]
            total, ntok = None, 0
            for x in acts[n]:
                loss, k = R.awq_clip_block_losses(w, x, w_amax, shrinks, m["block"])
                total = loss if total is None else total + loss
                ntok += k
            assert ntok == m["layers"][n]["num_tokens"], (name, n)
            assert torch.equal(total.reshape(len(shrinks), -1), t[f"{name}.{n}.losses"]), (name, n)
            best = R.awq_clip_best(total, w_amax, shrinks)
            assert bits_equal(best, t[f"{name}.{n}.best_clip"]), (name, n)
            assert bits_equal(t[f"{name}.{n}.amax"].reshape(best.shape), best), (name, n)


def test_mxfp8_oracle_matches_reference_compress():
    """oracle.mxfp8_quantize reproduces the reference's MXFP8QTensor.quantize (tests/golden/
    compress.*, written by running the reference's mtq.compress on the CPU) bit for bit."""
    import json

    from safetensors.torch import load_file

    t = load_file(str(G / "compress.safetensors"))
    meta = json.loads((G / "compress.json").read_text())
    for n in meta["mxfp8"]["linears"]:
        w = t[f"mxfp8.state.{n}.weight"]
        q, s = R.mxfp8_quantize(w)
        assert torch.equal(q.view(torch.uint8), t[f"mxfp8.q.{n}"]), n
        assert torch.equal(s, t[f"mxfp8.scale.{n}"]), n
