"""Accessors compatible with the reference's extension loaders (extensions.py:28-72).

``get_cuda_ext()`` / ``get_cuda_ext_fp8()`` / ``get_cuda_ext_mx()`` return objects exposing the
same functions as the reference's pybind modules (modelopt_cuda_ext: tensor_quant.cpp:63-76;
modelopt_cuda_ext_fp8: tensor_quant_gpu_fp8.cu:109-114; modelopt_cuda_ext_mx:
tensor_quant_mx.cu:393-411) -- backed by the MI355X-native library, so call sites written for the
reference's ext objects work unchanged.  They return ``None`` when the library is not built (and
``get_cuda_ext_mx(raise_if_failed=True)`` raises), like the reference.
"""

from __future__ import annotations

import enum
from types import SimpleNamespace

from modelopt_amd import _ext

__all__ = ["get_cuda_ext", "get_cuda_ext_fp8", "get_cuda_ext_mx", "precompile"]


class Types(enum.IntEnum):
    """Element/scale formats (tensor_quant_mx.h:38 ``enum class Types``)."""

    E4M3 = 0
    E5M2 = 1
    INT8 = 2
    E0M3 = 3
    E1M2 = 4
    E3M0 = 5
    E2M1 = 6
    E3M2 = 7
    E2M3 = 8
    E8M0 = 9


def _make(kind: str):
    ops = _ext.ops()
    if kind == "int":
        return SimpleNamespace(
            fake_tensor_quant=lambda inputs, amax, num_bits=8, unsigned=False, narrow_range=True: (
                ops.fake_tensor_quant(inputs, amax, num_bits, unsigned, narrow_range)
            ),
            fake_tensor_quant_=lambda inputs, amax, num_bits=8, unsigned=False, narrow_range=True: (
                ops.fake_tensor_quant_(inputs, amax, num_bits, unsigned, narrow_range)
            ),
            fake_tensor_quant_with_axis=lambda inputs, amax, axis, num_bits=8, unsigned=False, narrow_range=True: (
                ops.fake_tensor_quant_with_axis(inputs, amax, axis, num_bits, unsigned, narrow_range)
            ),
        )
    if kind == "fp8":
        return SimpleNamespace(
            fake_e4m3fy=lambda inputs, amax: ops.fake_e4m3fy(inputs, amax),
            fake_e4m3fy_with_axis=lambda inputs, amax, axis: ops.fake_e4m3fy_with_axis(inputs, amax, axis),
        )
    lib = _ext.kernel_cdll()
    return SimpleNamespace(
        Types=Types,
        fused_amax_convert=lambda inputs, block_size, format, scale_format, global_amax=None: (
            ops.fused_amax_convert(inputs, block_size, int(format), int(scale_format), global_amax)
        ),
        convert_to_exmy=lambda x, format: float(lib.mtq_convert_to_exmy(float(x), int(format))),
    )


def _get(kind: str, raise_if_failed: bool):
    cache = _get.__dict__.setdefault("cache", {})
    if kind not in cache:
        try:
            cache[kind] = _make(kind)
        except Exception:
            if raise_if_failed:
                raise
            cache[kind] = None
    return cache[kind]


def get_cuda_ext(raise_if_failed: bool = False):
    """INT fake-quant ext object (``modelopt_cuda_ext`` functions)."""
    return _get("int", raise_if_failed)


def get_cuda_ext_fp8(raise_if_failed: bool = False):
    """FP8 fake-quant ext object (``modelopt_cuda_ext_fp8`` functions)."""
    return _get("fp8", raise_if_failed)


def get_cuda_ext_mx(raise_if_failed: bool = False):
    """MX ext object (``modelopt_cuda_ext_mx`` functions)."""
    return _get("mx", raise_if_failed)


def precompile():
    """Build the in-tree libraries (the reference JIT-compiles here; we build ahead of time)."""
    import importlib.util
    import sys
    from pathlib import Path

    build_py = Path(__file__).resolve().parents[3] / "build.py"
    spec = importlib.util.spec_from_file_location("_mtq_build", build_py)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["_mtq_build"] = mod
    spec.loader.exec_module(mod)
    mod.build()
