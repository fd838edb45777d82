"""Loader for the in-tree MI355X-native libraries (``_lib/libmtq_amd.so`` and ``_lib/_C.so``).

The product has no CPU compute path and no fallback: if the HIP extension is missing, every
quantization op raises (``require_ops``).  The reference's equivalent loader silently returns
``None`` and falls back to ATen (modelopt/torch/utils/cpp_extension.py:57-96); here a missing
library is an error, so a run can never pass on a silent eager fallback.
"""

from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

import torch

LIB_DIR = Path(__file__).resolve().parent / "_lib"
KERNEL_LIB = LIB_DIR / "libmtq_amd.so"
OPS_LIB = LIB_DIR / "_C.so"
HEADER = Path(__file__).resolve().parents[2] / "include" / "mtq_amd.h"

_state: dict = {"ops": False, "cdll": None, "error": None}


class ExtensionMissingError(RuntimeError):
    """Raised when the MI355X-native extension is not built or cannot be loaded."""


def _load_ops() -> None:
    if _state["ops"]:
        return
    if not OPS_LIB.exists():
        raise ExtensionMissingError(
            f"modelopt_amd: {OPS_LIB} is missing; build it with "
            "`python tensorrt-model-optimizer_amd/build.py` (or __graft_entry__.build())"
        )
    torch.ops.load_library(str(OPS_LIB))
    _state["ops"] = True


def ops():
    """torch.ops.modelopt_amd, loading the op library on first use."""
    _load_ops()
    return torch.ops.modelopt_amd


def require_ops():
    return ops()


def is_available() -> bool:
    try:
        _load_ops()
        return True
    except Exception as e:  # noqa: BLE001
        _state["error"] = e
        return False


def kernel_cdll() -> ctypes.CDLL:
    """The C-ABI library itself (used for host-side helpers and the ABI symbol check)."""
    if _state["cdll"] is None:
        if not KERNEL_LIB.exists():
            raise ExtensionMissingError(f"modelopt_amd: {KERNEL_LIB} is missing")
        lib = ctypes.CDLL(str(KERNEL_LIB))
        lib.mtq_convert_to_exmy.restype = ctypes.c_float
        lib.mtq_convert_to_exmy.argtypes = [ctypes.c_float, ctypes.c_int]
        lib.mtq_status_string.restype = ctypes.c_char_p
        lib.mtq_status_string.argtypes = [ctypes.c_int]
        _state["cdll"] = lib
    return _state["cdll"]


def dispatch_counts() -> dict[str, int]:
    """Launches per kernel family since the library was loaded (``mtq_dispatch_counts``: the
    launchers pick vector / block-group / row-wave / persistent forms by shape; this shows which
    ones a workload reached).  Take two snapshots and subtract to scope it to a region."""
    _load_ops()  # the op library's copy of libmtq_amd.so is the one that launches
    lib = kernel_cdll()
    lib.mtq_dispatch_name.restype = ctypes.c_char_p
    lib.mtq_dispatch_name.argtypes = [ctypes.c_int]
    n = lib.mtq_dispatch_counts(None, 0)
    buf = (ctypes.c_int64 * n)()
    lib.mtq_dispatch_counts(buf, n)
    return {lib.mtq_dispatch_name(i).decode(): int(buf[i]) for i in range(n)}


def declared_symbols(header: Path = HEADER) -> list[str]:
    """Function names declared in include/mtq_amd.h."""
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mtq_[a-z0-9_]+)\s*\(", text)))


def loaded_library_paths() -> list[str]:
    """Paths of the in-tree .so files mapped into this process (for provenance checks)."""
    out = []
    try:
        with open(f"/proc/{os.getpid()}/maps") as f:
            for line in f:
                if str(LIB_DIR) in line:
                    p = line.split()[-1]
                    if p not in out:
                        out.append(p)
    except OSError:
        pass
    return out
