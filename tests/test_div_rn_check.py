"""The INT-n qdq division `mtq::div_rn` (csrc/mtq_device.hpp) equals IEEE `q / s`.

Runs a strided slice of the exhaustive host checker `scripts/check_div_rn.c` (the full sweep,
stride 1, is ~7.5e10 cases; its result is recorded in DESIGN.md).  The reference divides by the
scale: modelopt/torch/quantization/tensor_quant.py:643.
"""

import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_div_rn_matches_ieee_division(tmp_path):
    exe = tmp_path / "chk_div_rn"
    subprocess.run(
        ["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(REPO / "scripts" / "check_div_rn.c"), "-lm"],
        check=True,
    )
    r = subprocess.run([str(exe), "257"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert r.stdout.strip().endswith("mismatches 0"), r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_hist_division_matches_ieee_division(tmp_path):
    exe = tmp_path / "chk_hist"
    subprocess.run(
        ["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(REPO / "scripts" / "check_hist_division.c"), "-lm"],
        check=True,
    )
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert "mismatches 0" in r.stdout, r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_mxfp4_block_scale_division_matches_ieee(tmp_path):
    """The MXFP4 export's amax / 6 by div_rn (16-bit elements): every finite 16-bit amax."""
    exe = tmp_path / "chk_div6"
    subprocess.run(
        ["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(REPO / "scripts" / "check_div6.c"), "-lm"],
        check=True,
    )
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("mismatches 0"), r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_e8m0_exponent_shortcut(tmp_path):
    """mx_e8m0_exponent's fast path (mantissa > 64 -> ex + 1) equals ceil(fp32(log2(d)))
    (qtensor/mxfp4_tensor.py:62-66); strided slice of scripts/check_e8m0.c (stride 1 recorded in
    DESIGN §5)."""
    exe = tmp_path / "chk_e8m0"
    subprocess.run(
        ["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(REPO / "scripts" / "check_e8m0.c"), "-lm"],
        check=True,
    )
    r = subprocess.run([str(exe), "61"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert "mismatches 0" in r.stdout and "needing log2: 22" in r.stdout, r.stdout
