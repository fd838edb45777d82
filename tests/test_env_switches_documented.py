"""Every MTQ_AMD_* environment switch read by the sources is listed in DESIGN.md §8b (the table of
switches, their defaults and what they select), so A/B knobs cannot drift out of the docs."""

import re
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def test_every_env_switch_is_documented():
    pkg = REPO / "tensorrt-model-optimizer_amd"
    used = set()
    for path in list((pkg / "csrc").glob("*.hip")) + list((pkg / "csrc").glob("*.cpp")) + list(pkg.rglob("*.py")):
        used |= set(re.findall(r"MTQ_AMD_[A-Z0-9_]+", path.read_text(errors="ignore")))
    used.discard("MTQ_AMD_H_")  # header include guard, not a switch
    design = (REPO / "DESIGN.md").read_text()
    table = design[design.index("## 8b. Environment switches"):design.index("## 9. Status")]
    missing = sorted(u for u in used if u not in table)
    assert not missing, missing
    # at most 10 switches, each numerics or exercised by a test (the table says which);
    # no switch documented that the sources no longer read
    assert len(used) <= 10, sorted(used)
    documented = set(re.findall(r"`(MTQ_AMD_[A-Z0-9_]+)`", table)) - {"MTQ_AMD_DIST_BACKEND"}
    assert documented <= used, sorted(documented - used)


def test_awq_fused_switch_validated_at_use():
    """A misspelt MTQ_AMD_AWQ_FUSED warns at import (FP8 / max-only workflows still import) and
    makes awq_lite raise, before any calibration work."""
    import os
    import subprocess
    import sys

    env = {**os.environ, "MTQ_AMD_AWQ_FUSED": "alwyas",
           "PYTHONPATH": os.pathsep.join([str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)])}
    code = (
        "import torch, modelopt_amd.torch.quantization as mtq\n"
        "m = torch.nn.Linear(64, 64)\n"
        "mtq.quantize(m, mtq.INT8_DEFAULT_CFG, lambda mm: mm(torch.randn(4, 64)))\n"
        "print('max ok')\n"
        "mtq.quantize(torch.nn.Linear(64, 64), mtq.INT4_AWQ_CFG, lambda mm: mm(torch.randn(4, 64)))\n"
    )
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert "max ok" in r.stdout, r.stderr[-2000:]
    assert "MTQ_AMD_AWQ_FUSED='alwyas'" in r.stderr  # the import-time warning
    assert r.returncode != 0 and "ValueError: MTQ_AMD_AWQ_FUSED='alwyas'" in r.stderr, r.stderr[-2000:]
