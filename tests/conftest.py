"""Test configuration: markers, import paths, and GPU gating.

``-m "not gpu"`` runs here (no GPU): oracle-vs-golden, host logic, C-ABI symbol checks, gloo
multi-process logic.  ``-m gpu`` runs on an MI355X and exercises the HIP path through the C ABI /
torch ops, compared against the oracle (``oracle/``) and the golden fixtures.
"""

import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG_DIR = REPO / "tensorrt-model-optimizer_amd"
for p in (str(REPO), str(PKG_DIR)):
    if p not in sys.path:
        sys.path.insert(0, p)

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device) and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from modelopt_amd import _ext

    _ext.require_ops()  # fails loudly (not skip) when the extension is missing on a GPU box
    return torch.device("cuda:0")
