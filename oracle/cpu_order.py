"""Test infrastructure: ctypes access to ``oracle/awq_cpu_order.c`` (the host restatement of
ATen's CPU powf and column-sum order behind the AWQ-lite statistics; see that file).  Built by
``__graft_entry__.build()`` into ``oracle/_build/``; only ``tests/`` load it."""

from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SRC = HERE / "awq_cpu_order.c"
LIB = HERE / "_build" / "libawq_cpu_order.so"


def build(force: bool = False) -> Path:
    if force or not LIB.exists() or LIB.stat().st_mtime < SRC.stat().st_mtime:
        LIB.parent.mkdir(parents=True, exist_ok=True)
        tmp = LIB.with_suffix(".so.tmp")
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", str(SRC), "-o", str(tmp), "-lm"],
                       check=True)
        tmp.replace(LIB)
    return LIB


def _lib():
    lib = ctypes.CDLL(str(build()))
    f = ctypes.POINTER(ctypes.c_float)
    lib.oracle_powf_array.argtypes = [f, ctypes.c_int64, ctypes.c_float, f]
    lib.oracle_col_sum.argtypes = [f, ctypes.c_int64, ctypes.c_int64, f]
    return lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def powf(x: np.ndarray, y: float) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    _lib().oracle_powf_array(_ptr(x), x.size, ctypes.c_float(y), _ptr(out))
    return out


def col_sum(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32)
    out = np.empty(a.shape[1], dtype=np.float32)
    _lib().oracle_col_sum(_ptr(a), a.shape[0], a.shape[1], _ptr(out))
    return out
