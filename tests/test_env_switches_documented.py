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
