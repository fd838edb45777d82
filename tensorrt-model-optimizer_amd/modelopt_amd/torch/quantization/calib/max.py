"""Max calibrator on the fused accumulate-max HIP kernel.

Reference: modelopt/torch/quantization/calib/max.py:26-110.  Same results (the running amax is an
exact max, so order and fusion cannot change it); the differences are where the time goes:

* one kernel launch per ``collect`` (``amax_accumulate``: max|x| folded straight into a persistent
  fp32 running-max buffer) instead of ``reduce_amax``'s two full passes plus ``torch.max``;
* no host synchronisation in ``collect``: the reference's three NaN / negative / inf asserts
  (calib/max.py:69-77) are evaluated once, lazily, when the amax is read (``compute_amax``), and
  raise the same AssertionError messages there;
* a second ``collect`` of the *same* data at the same version -- the same tensor object, or the
  same view (offset/shape/stride) of the same live base tensor (the weight of a QuantLinear, or
  one expert's slice of a fused [E, N, K] expert weight, during ``forward_loop``, which the
  reference re-reduces on every batch) -- is skipped: max(a, a) = a.  The skip holds only
  within one collection epoch (``enable_stats_collection`` opens a new one), because writes
  through ``.data`` (weight folding between calibration passes) do not bump ``_version``;
  inference tensors (no version counter) are never skipped.
"""

from __future__ import annotations

import weakref

import torch

from ..utils import core_utils as quant_utils
from .calibrator import _Calibrator

__all__ = ["MaxCalibrator"]

# The last tensor reduced by a calibrator: (weakref to its base, (view key, _version, reduce
# axes), weakref to the calibrator, its per-call amax buffer or None).  See _accumulate.
_SHARED = None
# Collection epoch: bumped by ``new_collect_epoch`` (called from ``enable_stats_collection``).
_EPOCH = 0


def _ops():
    from modelopt_amd._ext import ops

    return ops()


def _zeros_f32(numel: int, device) -> torch.Tensor:
    """A zeroed fp32 running-max buffer.  On the GPU the fill is the kernel library's own, so a
    calibration pass launches no torch kernel the model's forward has not loaded (the first launch
    from a code object not loaded yet stalls the host for tens to hundreds of ms)."""
    if torch.device(device).type != "cuda":
        return torch.zeros(numel, dtype=torch.float32, device=device)
    t = torch.empty(numel, dtype=torch.float32, device=device)
    _ops().amax_fill_(t, 0.0)
    return t


def _fold_max(dst: torch.Tensor, src: torch.Tensor) -> None:
    """dst = max(dst, src) (NaN propagates), the library's kernel on the GPU (see _zeros_f32)."""
    if dst.is_cuda:
        _ops().amax_fold_(dst, src)
    else:
        torch.maximum(dst, src, out=dst)


def _bad_flags(x: torch.Tensor) -> torch.Tensor:
    """int32 [3] on x's device: any NaN, any +-inf, any negative value (one launch on the GPU)."""
    if x.is_cuda:
        return _ops().amax_check(x)
    return torch.stack([torch.isnan(x).any(), torch.isinf(x).any(), (x < 0).any()]).to(torch.int32)


def new_collect_epoch() -> None:
    """Forget every calibrator's "same tensor as last collect" key (``.data`` writes between
    calibration passes do not bump ``_version``, so a key may not outlive its pass)."""
    global _EPOCH, _SHARED
    _EPOCH += 1
    _SHARED = None


def quantizer_call_is_noop(q, x) -> bool:
    """True when calling the TensorQuantizer ``q`` on ``x`` would return ``x`` unchanged and do
    nothing else: collect-only (max calibration, no fake quant), no pre_quant_scale, no block
    reshape, and a MaxCalibrator that has just collected this very tensor view at this version (so
    its collect is skipped).  Lets hot callers (a weight quantizer on every forward of a max
    calibration pass) skip the module call entirely."""
    d = q.__dict__
    if not d.get("_if_calib") or d.get("_if_quant") or d.get("_disabled") or d.get("_dynamic"):
        return False
    if d.get("_block_sizes") is not None or q.pre_quant_scale is not None:
        return False
    cal = d.get("_calibrator")
    return type(cal) is MaxCalibrator and cal._acc is not None and cal._same_as_last(x)


class MaxCalibrator(_Calibrator):
    """Tracks the absolute max of all collected tensors (per-tensor or along ``axis``)."""

    def __init__(self, num_bits=8, axis=None, unsigned=False, track_amax=False):
        super().__init__(num_bits, axis, unsigned)
        self._track_amax = track_amax
        if self._track_amax:
            self._amaxs = []
        self._acc = None  # fp32 running max, flat
        self._out_shape = None
        self._out_dtype = None
        self._last = None  # (weakref to the base of the last collected tensor, view key, _version)
        self._meta_amax = None
        self._validated = False  # NaN/inf checks done for the current running max
        self._share = False  # another calibrator collects the same tensors: publish results
        self._tmp = None

    @property
    def amaxs(self):
        return self._amaxs

    @staticmethod
    def _view_key(x):
        base = x._base if x._base is not None else x
        return base, (x.storage_offset(), tuple(x.shape), x.stride(), x.dtype)

    def _same_as_last(self, x, vk=None) -> bool:
        if self._last is None:
            return False
        ref, key, ver, epoch = self._last
        if epoch != _EPOCH or x.is_inference():
            return False
        base, k = self._view_key(x) if vk is None else vk
        return ref() is base and k == key and x._version == ver

    def collect(self, x):
        # calibration forwards run under no_grad already: enter the context only when needed
        # (the decorator form costs several microseconds per call, on every quantizer call)
        if torch.is_grad_enabled():
            with torch.no_grad():
                return self._collect(x)
        return self._collect(x)

    def _collect(self, x):
        reduce_axis = None if self._axis is None else quant_utils.convert_quantization_axis_to_reduce_axis(x, self._axis)
        if x.is_meta:
            self._meta_amax = quant_utils.amax_view(x, reduce_axis)[4]
            return
        vk = None if x.is_inference() else self._view_key(x)
        if self._acc is not None and vk is not None and self._same_as_last(x, vk):
            return
        keep_shape = quant_utils.amax_view(x, reduce_axis)[4] if reduce_axis is not None else []
        if self._acc is None:
            numel = 1
            for s in keep_shape:
                numel *= s
            self._acc = _zeros_f32(numel, x.device)
            self._out_shape = keep_shape
            self._out_dtype = x.dtype if x.dtype.is_floating_point else torch.float32
            if self._out_dtype in (torch.float8_e4m3fn, torch.float8_e5m2):
                self._out_dtype = torch.get_default_dtype()
        elif list(keep_shape) != list(self._out_shape):
            raise RuntimeError("amax shape changed!")
        self._validated = False
        base = None
        self._last = None
        if vk is not None:  # inference tensors have no version counter
            try:
                base, key = vk
                self._last = (weakref.ref(base), key, x._version, _EPOCH)
            except TypeError:
                base = None
        self._accumulate(x, reduce_axis, base)
        if self._track_amax:
            self._amaxs.append(quant_utils.reduce_amax(x, axis=reduce_axis).cpu().numpy())

    def _accumulate(self, x, reduce_axis, base):
        """Fold max|x| into the running max, sharing one reduction between calibrators that
        collect the very same tensor: q/k/v_proj (and gate/up_proj) input quantizers all see
        the one normalised hidden state, so the reference reduces it 3 (2) times per layer and
        batch.  The first calibrator to see a tensor records it; a sibling that then sees the
        same tensor marks the first one as a *producer*, which from the next batch on reduces
        into a private buffer that the siblings fold in with one elementwise max.  max is exact
        and order-free, so every running max is bit-identical to an unshared collect."""
        global _SHARED
        if base is None or self._track_amax:
            quant_utils.reduce_amax_accumulate(x, self._acc, reduce_axis)
            return
        key = (self._last[1], x._version, None if reduce_axis is None else tuple(reduce_axis))
        entry = _SHARED
        if entry is not None and entry[0]() is base and entry[1] == key and entry[2]() is not self:
            result = entry[3]
            if result is not None and result.numel() == self._acc.numel():
                _fold_max(self._acc, result)
                return
            producer = entry[2]()
            if producer is not None:
                producer._share = True
            quant_utils.reduce_amax_accumulate(x, self._acc, reduce_axis)
            return
        if getattr(self, "_share", False):
            if self._tmp is None or self._tmp.numel() != self._acc.numel():
                self._tmp = torch.empty_like(self._acc)
            if self._tmp.is_cuda:
                _ops().amax_fill_(self._tmp, 0.0)
            else:
                self._tmp.zero_()
            quant_utils.reduce_amax_accumulate(x, self._tmp, reduce_axis)
            _fold_max(self._acc, self._tmp)
            _SHARED = (weakref.ref(base), key, weakref.ref(self), self._tmp)
        else:
            quant_utils.reduce_amax_accumulate(x, self._acc, reduce_axis)
            _SHARED = (weakref.ref(base), key, weakref.ref(self), None)

    def _result(self):
        if self._acc is None:
            return None
        out = self._acc.view(self._out_shape) if self._out_shape else self._acc.view(())
        out = out.to(self._out_dtype)
        if out.numel() == 1:
            out = out.squeeze()
        return out

    @property
    def _calib_amax(self):
        return self._result()

    def reset(self):
        global _SHARED
        self._acc = None
        self._out_shape = None
        self._last = None
        self._validated = False
        self._tmp = None
        if _SHARED is not None and _SHARED[2]() is self:
            _SHARED = None

    def validate(self):
        """The reference's per-collect asserts (calib/max.py:69-77), evaluated once."""
        if self._acc is None or self._validated:
            return
        bad = _bad_flags(self._acc).tolist()
        assert not bad[0], "detected nan values in amax (NaN in a collected tensor)"
        assert not bad[1], "detected inf values in amax (inf in a collected tensor)"
        self._validated = True

    @staticmethod
    def validate_many(calibrators) -> None:
        """Batched ``validate`` for many calibrators: one concatenated NaN/inf check (one host
        sync per device) instead of one per quantizer (448 for Llama-3-8B FP8).  Clean
        calibrators are marked validated; if any running max holds NaN/inf, each calibrator is
        left to raise its own AssertionError in ``compute_amax``."""
        by_dev: dict = {}
        for c in calibrators:
            if isinstance(c, MaxCalibrator) and c._acc is not None and not c._validated:
                by_dev.setdefault(c._acc.device, []).append(c)
        for cs in by_dev.values():
            flags = _bad_flags(torch.cat([c._acc for c in cs])).tolist()
            if not (flags[0] or flags[1]):
                for c in cs:
                    c._validated = True

    def compute_amax(self):
        self.validate()
        return self._result()

    def __str__(self):
        return f"MaxCalibrator(track_amax={self._track_amax})"

    def __repr__(self):
        return f"MaxCalibrator({super().__repr__()} calib_amax={self._result()} track_amax={self._track_amax})"
