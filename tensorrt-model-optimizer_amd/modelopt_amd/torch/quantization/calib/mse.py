"""MSE amax calibrators (reference: modelopt/torch/quantization/calib/mse.py:31-300).

Same classes, arguments, candidate sets and selection rule as the reference.  What changes is
how ``collect`` evaluates the candidates on MI355X:

* ``MseCalibrator`` (multiplier search, 39 candidates by default): when ``quant_func`` is the
  weight quantizer's own ``_mse_quant_func`` and that quantizer is an INT-n / E4M3 fake quantizer
  with a per-tensor, per-row or static-block amax, all candidates are evaluated by ONE HIP pass
  (``torch.ops.modelopt_amd.mse_sweep``: the weight is read once, every candidate's qdq and
  squared error are computed in registers) instead of the reference's per-candidate
  quantize + mse_loss + reduce (three full-tensor passes per candidate).  Any other quant_func
  runs the reference loop on the device with the quantizer's HIP kernels.
* ``NVFP4MSECalibrator`` (126 FP8 scale candidates): the fused sweep is
  ``torch.ops.modelopt_amd.nvfp4_fp8_scale_sweep`` (the reference's Triton
  ``nvfp4_fp8_scale_sweep``), bit-identical to it.  ``MODELOPT_NVFP4_TRITON_SWEEP=0`` selects the
  reference's 126-step loop, as in the reference.

The 126 candidates are ``E4M3 value / 448`` formed with a true fp32 division (the CPU reference's
arithmetic).  On CUDA the reference builds them on the device, where torch divides by a CPU scalar
as a multiply by its reciprocal (1 ulp off for 76 of the 126); DESIGN.md §4c.
"""

from __future__ import annotations

import math
import os
from collections.abc import Callable

import torch
import torch.nn.functional as F

from .. import utils as quant_utils
from .calibrator import _Calibrator

__all__ = ["MseCalibrator", "NVFP4MSECalibrator", "fp8_scale_candidates"]

_CAND_CACHE: dict = {}


def fp8_scale_candidates(device: torch.device | str = "cpu") -> torch.Tensor:
    """The 126 finite positive E4M3 values / 448 (reference _fp8_scale_candidates.py:25-32)."""
    dev = torch.device(device)
    c = _CAND_CACHE.get(dev)
    if c is None:
        u = torch.arange(0, 128, dtype=torch.uint8).view(torch.float8_e4m3fn).float()
        c = (u[torch.isfinite(u) & (u > 0)] / 448.0).to(dev)  # divided on the host: RN(v / 448)
        _CAND_CACHE[dev] = c
    return c


def _ops():
    from modelopt_amd._ext import ops

    return ops()


def _fused_mse_plan(x: torch.Tensor, initial_amax: torch.Tensor, axis, quant_func):
    """(x2d, amax, num_bits, unsigned, narrow, round_amax) when the fused sweep reproduces
    ``quant_func(x, initial_amax * c)`` exactly, else None."""
    from ..nn.modules.tensor_quantizer import TensorQuantizer

    q = getattr(quant_func, "keywords", {}).get("quantizer") if hasattr(quant_func, "func") else None
    if q is None or getattr(quant_func.func, "__name__", "") != "_mse_quant_func":
        return None
    if not isinstance(q, TensorQuantizer) or type(q).__name__ not in ("TensorQuantizer", "StaticBlockScaleQuantizer"):
        return None
    if not x.is_cuda or x.dtype not in (torch.float32, torch.float16, torch.bfloat16):
        return None
    if q.backend is not None or not q.fake_quant or q.pre_quant_scale is not None or q.is_mx_format:
        return None
    if getattr(q, "is_nvfp4_static", False) or (q.block_sizes or {}).get("type") == "dynamic":
        return None
    if hasattr(q, "_bias_value") or getattr(q, "_use_constant_amax", False):
        return None
    nb = q._num_bits
    if isinstance(nb, tuple):
        if tuple(nb) != (4, 3):
            return None
        bits, uns, narrow = 0, False, False
    elif isinstance(nb, int) and 1 <= nb <= 16:
        bits, uns, narrow = nb, bool(q._unsigned), bool(q._narrow_range)
    else:
        return None
    if initial_amax.numel() == 1 and axis is None:
        x2 = x.reshape(1, -1)
    elif axis in (0, (0,), [0]) and x.dim() == 2 and initial_amax.numel() == x.shape[0]:
        x2 = x
    else:
        return None
    if x2.shape[1] > 128 and x2.shape[0] > 65535:
        return None
    return x2, initial_amax, bits, uns, narrow, initial_amax.dim() != 0


class MseCalibrator(_Calibrator):
    """Per-tensor / per-channel MSE amax search (reference calib/mse.py:31-183)."""

    def __init__(
        self,
        amax: torch.Tensor,
        axis: int | tuple | list | None = None,
        step_size: float = 0.1,
        start_multiplier: float = 0.25,
        stop_multiplier: float = 4.0,
        quant_func: Callable[[torch.Tensor, torch.Tensor], torch.Tensor] | None = None,
        error_func: Callable[[torch.Tensor, torch.Tensor], torch.Tensor] | None = None,
    ):
        super().__init__(num_bits=None, axis=axis, unsigned=None)
        self._initial_amax = amax
        self._step_size = step_size
        self._start_multiplier = start_multiplier
        self._stop_multiplier = stop_multiplier
        self._num_steps = math.ceil((stop_multiplier - start_multiplier) / step_size) + 1
        self._quant_func = quant_func
        self._error_func = error_func
        self._losses_sum: list[torch.Tensor | None] | None = None
        self._candidates: torch.Tensor | None = None
        self._amax: torch.Tensor | None = None

    def _generate_candidates(self, device: torch.device) -> torch.Tensor:
        return torch.linspace(self._start_multiplier, self._stop_multiplier, steps=self._num_steps, device=device)

    def _compute_candidate_amax(self, candidates: torch.Tensor) -> torch.Tensor:
        if candidates.ndim != 0:  # final compute_amax
            candidates = candidates.view_as(self._initial_amax)
        return self._initial_amax * candidates

    def _add_losses(self, step: int, loss: torch.Tensor):
        if self._losses_sum[step] is None:
            self._losses_sum[step] = loss.clone()
        else:
            self._losses_sum[step] += loss

    @torch.no_grad()
    def collect(self, x: torch.Tensor):
        if self._quant_func is None:
            raise RuntimeError("Quantization function not set.")
        device = x.device
        candidates = self._generate_candidates(device)
        if self._candidates is None:
            self._candidates = candidates
            self._num_steps = len(candidates)
            self._losses_sum = [None] * self._num_steps
        assert self._losses_sum is not None
        plan = None
        if self._error_func is None and type(self)._compute_candidate_amax is MseCalibrator._compute_candidate_amax:
            plan = _fused_mse_plan(x.detach(), self._initial_amax, self._axis, self._quant_func)
        if plan is not None:
            x2, amax, bits, uns, narrow, round_amax = plan
            losses = _ops().mse_sweep(x2.detach(), amax, candidates.float(), bits, uns, narrow, round_amax)
            per_tensor = self._axis is None
            for step in range(self._num_steps):
                self._add_losses(step, losses[step].reshape(()) if per_tensor else losses[step])
            return
        x = x.detach().to(dtype=torch.float32)
        reduce_axis = quant_utils.convert_quantization_axis_to_reduce_axis(x, self._axis)
        for step, candidate in enumerate(candidates):
            xq = self._quant_func(x, self._compute_candidate_amax(candidate))
            error = self._error_func(x, xq) if self._error_func is not None else F.mse_loss(x, xq, reduction="none")
            self._add_losses(step, quant_utils.reduce_sum(error, axis=reduce_axis, keepdims=False))

    def reset(self):
        self._losses_sum = None
        self._candidates = None
        self._amax = None
        if self._initial_amax is not None:
            del self._initial_amax
            self._initial_amax = None

    @torch.no_grad()
    def compute_amax(self, verbose: bool = False):
        if self._losses_sum is None or not any(loss is not None for loss in self._losses_sum):
            return None
        first = next(loss for loss in self._losses_sum if loss is not None)
        losses = []
        for step in range(self._num_steps):
            if self._losses_sum[step] is not None:
                losses.append(self._losses_sum[step])
            elif first.ndim == 0:
                losses.append(torch.tensor(float("inf"), device=first.device))
            else:
                losses.append(torch.full_like(first, float("inf")))
        best = torch.argmin(torch.stack(losses), dim=0)
        assert self._candidates is not None
        self._amax = self._compute_candidate_amax(self._candidates[best])
        if verbose:
            ratio = self._amax / self._initial_amax
            if ratio.ndim == 0:
                print(f"MSE Calibrator: best_amax/initial_amax ratio = {ratio.item():.4f}")
            else:
                print(
                    f"MSE Calibrator: best_amax/initial_amax ratio - mean: {ratio.mean().item():.4f}, "
                    f"min: {ratio.min().item():.4f}, max: {ratio.max().item():.4f}"
                )
        return self._amax


class NVFP4MSECalibrator(MseCalibrator):
    """Per-block FP8-scale sweep for NVFP4 static weights (reference calib/mse.py:186-300).

    One-shot between resets, like the reference: ``collect`` caches the final per-block amax.
    The Hessian-weighted sweep (local_hessian) is outside the MI355X path."""

    def __init__(
        self,
        amax: torch.Tensor,
        global_amax: torch.Tensor,
        axis: int | tuple | list | None = None,
        quant_func: Callable | None = None,
        error_func: Callable | None = None,
        hessian: torch.Tensor | None = None,
    ):
        super().__init__(amax=amax, axis=axis, quant_func=quant_func, error_func=error_func)
        self._global_amax = global_amax.to(dtype=torch.float32)
        self._hessian = hessian
        self._best_amax: torch.Tensor | None = None

    def _compute_candidate_amax(self, candidates: torch.Tensor) -> torch.Tensor:
        if candidates.ndim != 0:
            candidates = candidates.view_as(self._initial_amax)
        return torch.ones_like(self._initial_amax, dtype=torch.float32) * (self._global_amax * candidates)

    def _generate_candidates(self, device: torch.device) -> torch.Tensor:
        return fp8_scale_candidates(device)

    def _sweep_eligible(self, x: torch.Tensor) -> bool:
        return (
            x.is_cuda
            and os.environ.get("MODELOPT_NVFP4_TRITON_SWEEP", "1") != "0"
            and self._initial_amax is not None
            and x.ndim == 2
            and x.shape[0] == int(self._initial_amax.numel())
            and x.shape[1] in (8, 16, 32)
            and x.dtype in (torch.float32, torch.float16, torch.bfloat16)
        )

    @torch.no_grad()
    def collect(self, x: torch.Tensor):
        if self._best_amax is not None:
            raise RuntimeError(
                "NVFP4MSECalibrator: a previous collect() call produced a final amax; "
                "multi-collect is not supported. Call reset() to start a fresh cycle."
            )
        if self._hessian is not None:
            raise NotImplementedError("modelopt_amd: the Hessian-weighted NVFP4 sweep (local_hessian) is out of scope")
        if self._error_func is None and self._sweep_eligible(x):
            best = _ops().nvfp4_fp8_scale_sweep(
                x.detach(), self._global_amax, fp8_scale_candidates(x.device), x.shape[-1]
            )
            self._best_amax = best.reshape(self._initial_amax.shape).to(dtype=torch.float32)
            return
        self._run_reference_collect(x)

    def _run_reference_collect(self, x: torch.Tensor):
        super().collect(x)
        best = super().compute_amax(verbose=False)
        self._best_amax = best.to(dtype=torch.float32) if best is not None else None
        self._losses_sum = None

    @torch.no_grad()
    def compute_amax(self, verbose: bool = False):
        return self._best_amax

    def reset(self):
        self._best_amax = None
        self._losses_sum = None
        self._candidates = None
        self._amax = None
