"""Reduction helpers of the quantization hot path on the HIP kernels.

Mirrors modelopt/torch/quantization/utils/core_utils.py:128-183 (``reduce_amax``,
``convert_quantization_axis_to_reduce_axis``).  ``reduce_amax`` is one launch of the
``amax_accumulate`` kernel (max|x| with NaN propagation) instead of the reference's two full
passes (``torch.max`` + ``torch.min``); the value and dtype are identical.
"""

from __future__ import annotations

import contextlib
import gc

import torch

from modelopt_amd._ext import ops as _ext_ops

_FP8_DTYPES = tuple(
    d for d in (getattr(torch, "float8_e4m3fn", None), getattr(torch, "float8_e5m2", None)) if d
)
_KERNEL_DTYPES = (torch.float32, torch.float16, torch.bfloat16)

__all__ = [
    "amax_view",
    "convert_quantization_axis_to_reduce_axis",
    "reduce_amax",
    "reduce_amax_accumulate",
    "reduce_sum",
]


def convert_quantization_axis_to_reduce_axis(input, axis):
    """Quantization axis -> axes to reduce (None = all); core_utils.py:128-143."""
    if axis is None:
        return None
    axis = axis if isinstance(axis, (list, tuple)) else [axis]
    return [i for i in range(input.dim()) if i not in axis and (i - input.dim()) not in axis]


def _norm_axes(axis, ndim):
    if isinstance(axis, int):
        axis = (axis,)
    return sorted({a + ndim if a < 0 else a for a in axis})


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense (the elements fill one contiguous storage range)."""
    if t.numel() == 0:
        return False
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz != 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


def amax_view(input: torch.Tensor, reduce_axis) -> tuple[torch.Tensor, int, int, int, list[int]]:
    """Map a reduction to the kernel's [P, K, Q] view.

    Returns ``(x, P, K, Q, keep_shape)`` where ``x`` is contiguous with the kept axes forming one
    contiguous run (the input is permuted only when the kept axes are not adjacent) and
    ``keep_shape`` is the keepdims output shape.
    """
    nd = input.dim()
    if reduce_axis is None and not input.is_contiguous() and _dense(input):
        # per-tensor max is layout-free: read a dense strided tensor in storage order
        return input.as_strided((input.numel(),), (1,)), 1, 1, input.numel(), [1] * nd
    if reduce_axis is None:
        red = list(range(nd))
    else:
        red = _norm_axes(reduce_axis, nd)
    keep = [d for d in range(nd) if d not in red]
    keep_shape = [1 if d in red else input.shape[d] for d in range(nd)]
    x = input
    if keep and keep != list(range(keep[0], keep[-1] + 1)):
        # non-adjacent kept axes: move them together (rare; a device-side permute copy)
        perm = red[: sum(1 for r in red if r < keep[0])] + keep
        perm += [d for d in range(nd) if d not in perm]
        x = x.permute(perm)
        keep_pos = list(range(perm.index(keep[0]), perm.index(keep[0]) + len(keep)))
        sizes = list(x.shape)
    else:
        keep_pos = keep
        sizes = list(x.shape)
    x = x.contiguous()
    if not keep_pos:
        return x, 1, 1, max(x.numel(), 0), keep_shape
    a, b = keep_pos[0], keep_pos[-1]
    P = 1
    for s in sizes[:a]:
        P *= s
    K = 1
    for s in sizes[a : b + 1]:
        K *= s
    Q = 1
    for s in sizes[b + 1 :]:
        Q *= s
    return x, P, K, Q, keep_shape


def reduce_amax_accumulate(input: torch.Tensor, out: torch.Tensor, reduce_axis=None) -> None:
    """``out = max(out, max|input|)`` over ``reduce_axis`` (fp32 ``out``, one kernel launch).

    This is the running-max accumulator of ``MaxCalibrator.collect`` (calib/max.py:53-86) fused
    with ``reduce_amax``: no intermediate amax tensor, no host-side NaN/inf asserts.
    """
    if reduce_axis is None and input.dtype in _KERNEL_DTYPES and input.is_contiguous():
        # per-tensor max of a contiguous tensor (the common activation collect): no view mapping
        n = input.numel()
        if n:
            _amax_op()(input, out if out.dim() == 1 else out.view(-1), 1, 1, n)
        return
    if input.dtype in _FP8_DTYPES:
        input = input.to(torch.get_default_dtype())
    x, P, K, Q, _ = amax_view(input, reduce_axis)
    if x.numel() == 0:
        return
    if x.dtype not in _KERNEL_DTYPES:
        # float64 has no HIP reduction kernel (fp32 accumulation would round it)
        raise TypeError(f"modelopt_amd: amax reduction does not support {x.dtype}")
    _amax_op()(x, out.view(-1), P, K, Q)


_AMAX_OP = []


def _amax_op():
    """The amax_accumulate OpOverload, resolved once (the packet lookup and overload resolution
    of ``torch.ops.modelopt_amd.amax_accumulate`` cost microseconds on every collect)."""
    if not _AMAX_OP:
        _AMAX_OP.append(_ext_ops().amax_accumulate.default)
    return _AMAX_OP[0]


@torch.no_grad()
def reduce_amax(input, axis=None, keepdims=True, squeeze_scalar=True):
    """Absolute max over ``axis`` (the reduce axes), same value/shape/dtype as the reference."""
    if input.dtype in _FP8_DTYPES:
        input = input.to(torch.get_default_dtype())
    if input.dtype == torch.float64:
        raise TypeError("modelopt_amd: amax reduction does not support float64")
    if axis is None:
        out = torch.zeros((), dtype=torch.float32, device=input.device)
        reduce_amax_accumulate(input, out, None)
        return out.to(input.dtype)
    if isinstance(axis, int):
        axis = (axis,)
    _, _, K, _, keep_shape = amax_view(input, axis)
    out = torch.zeros(K, dtype=torch.float32, device=input.device)
    reduce_amax_accumulate(input, out, axis)
    red = _norm_axes(axis, input.dim())
    if keepdims:
        out = out.view(keep_shape)
    else:
        out = out.view([s for d, s in enumerate(input.shape) if d not in red])
    out = out.to(input.dtype)
    if squeeze_scalar and out.numel() == 1:
        out.squeeze_()
    return out


def reduce_sum(input, axis=None, keepdims=True):
    """Sum over ``axis`` (all dims when None) -- reference core_utils.py:187-212."""
    if axis is None:
        return torch.sum(input)
    if isinstance(axis, int):
        axis = (axis,)
    return torch.sum(input, dim=axis, keepdim=keepdims)


@contextlib.contextmanager
def gc_paused():
    """Pause Python's cyclic GC around bookkeeping that allocates many small objects next to a
    large model heap (conversion, amax loading): a generation-2 collection triggered there cost
    0.16 s of a 0.26 s Llama-3-8B conversion on the GPU box.  Collections resume on exit."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def update_quant_cfg_with_kv_cache_quant(quant_cfg: dict, kv_cache_quant_cfg: list) -> dict:
    """A deep copy of ``quant_cfg`` with the KV-cache entries (e.g. ``FP8_KV_CFG["quant_cfg"]``)
    appended to its ``quant_cfg`` list -- an empty / missing list starts from "disable every
    quantizer" -- and ``algorithm`` defaulted to ``"max"`` (reference utils/core_utils.py:1049-1075)."""
    import copy as _copy

    out = _copy.deepcopy(quant_cfg)
    inner = out.get("quant_cfg") or [{"quantizer_name": "*", "enable": False}]
    out["quant_cfg"] = list(inner) + _copy.deepcopy(list(kv_cache_quant_cfg))
    if not out.get("algorithm"):
        out["algorithm"] = "max"
    return out

