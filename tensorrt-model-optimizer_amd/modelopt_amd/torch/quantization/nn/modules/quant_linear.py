"""Quantized Linear (reference: nn/modules/quant_linear.py:38-53).

MI355X addition: for short inputs (<= 16 rows after flattening, decode / small-batch evaluation
of a quantized model) the forward runs the fused MFMA kernel ``qlinear_small_m``, which applies
the weight fake quant to the GEMM operands in registers instead of writing a dequantised copy of
the weight to HBM and reading it back (one pass over W instead of three).  The dequantised weight
values are bit-identical to the unfused path (same qdq helpers); only the GEMM summation order
differs.  Gradients, calibration, dynamic / MX / NVFP4 / custom-backend weight quantizers and
long inputs take the reference's path.  ``MTQ_AMD_FUSED_QLINEAR=0`` disables the fusion.
"""

import os

import torch
import torch.nn as nn

from modelopt_amd._ext import ops as _ops

from ... import tensor_quant
from .quant_module import QuantLinearConvBase, QuantModuleRegistry
from .tensor_quantizer import StaticBlockScaleQuantizer, TensorQuantizer

__all__ = ["Linear", "QuantLinear"]

_FUSED_MAX_ROWS = 16
_FUSED = [os.environ.get("MTQ_AMD_FUSED_QLINEAR", "1") != "0"]


def _fused_weight_params(wq, weight):
    """(amax, block, kind) when ``wq``'s fake quant of ``weight`` is an element-wise INT-n / FP8
    qdq with a per-tensor, per-output-channel or 1-D static-block (along K) amax; else None."""
    if type(wq) not in (TensorQuantizer, StaticBlockScaleQuantizer):
        return None
    if wq._disabled or not wq._if_quant or wq._if_calib or not wq._fake_quant or wq._dynamic:
        return None
    if wq.backend is not None or wq.pre_quant_scale is not None or wq.is_mx_format:
        return None
    if isinstance(wq, StaticBlockScaleQuantizer) and wq.is_nvfp4_static:
        return None
    amax = getattr(wq, "_amax", None)
    if amax is None or amax.device != weight.device or amax.numel() < 1:
        return None
    nb = wq._num_bits
    if nb == (4, 3):
        kind = 1
    elif isinstance(nb, int) and not isinstance(nb, bool):
        kind = 0
    else:
        return None
    n, k = weight.shape
    bs = wq._block_sizes
    if amax.numel() == 1:
        return amax, k, kind
    if not bs and amax.numel() == n and tuple(amax.shape) in ((n, 1), (n,)):
        return amax, k, kind  # per output channel (axis 0)
    if bs and set(bs) <= {-1, 1, "type"} and bs.get("type", "static") == "static":
        b = bs.get(-1) or bs.get(1)
        if b and k % b == 0 and b % 32 == 0 and amax.numel() * b == n * k:
            return amax, b, kind
    return None


def _fused_params(mod, input):
    """(weight, bias, (amax, block, kind)) when ``mod`` can run the fused short-input forward on
    ``input``; None otherwise.  No side effects (the input quantizer is not applied)."""
    if not _FUSED[0] or input.device.type != "cuda" or input.dtype not in (torch.bfloat16, torch.float16):
        return None
    weight = mod._parameters.get("weight")
    if weight is None or weight.dtype != input.dtype or weight.dim() != 2:
        return None
    if not weight.is_contiguous() or weight.data_ptr() % 16:
        return None  # a view into a fused / tied parameter: the kernel streams 16-byte vectors
    n, k = weight.shape
    if input.shape[-1] != k or k % 32 or n % 16 or input.numel() // max(k, 1) > _FUSED_MAX_ROWS:
        return None
    if torch.is_grad_enabled() and (input.requires_grad or weight.requires_grad):
        return None
    wq, oq = mod._modules.get("weight_quantizer"), mod._modules.get("output_quantizer")
    if oq is not None and oq.is_enabled:
        return None
    p = _fused_weight_params(wq, weight)
    if p is None:
        return None
    bias = mod._parameters.get("bias")
    if bias is not None and bias.dtype != input.dtype:
        return None
    return weight, bias, p


def _fused_input(mod, input):
    x = mod.input_quantizer(input)
    if x.dtype != input.dtype:
        return None
    x = x.contiguous()
    if x.data_ptr() % 16:
        x = x.clone()  # the MFMA operand loads are 16-byte vectors
    return x


def _fused_forward(mod, input):
    """The fused short-input forward, or None when the module/input does not qualify."""
    fp = _fused_params(mod, input)
    if fp is None:
        return None
    weight, bias, (amax, block, kind) = fp
    x = _fused_input(mod, input)
    if x is None:
        return None
    wq = mod._modules["weight_quantizer"]
    return _ops().qlinear_small_m(
        x, weight, bias, amax, block, kind, wq._num_bits if kind == 0 else 8, bool(wq._unsigned),
        bool(wq._narrow_range),
    )


def _input_quantizer_pure(mod) -> bool:
    """The module's input quantizer is a plain function of its input: no calibration collect."""
    q = mod._modules.get("input_quantizer")
    if q is None:
        return True
    if type(q) is not TensorQuantizer:
        return False
    return q._disabled or not q._if_calib


class ProjectionGroup:
    """The projections of one attention forward that read the same hidden state (q/k/v_proj):
    the first of them to be called with a short input runs all of them as ONE launch
    (``qlinear_small_m_group``) and hands the others their outputs when they are called with the
    same tensor.  Each input quantizer is still applied exactly once, each output is what that
    projection's own fused forward computes (only the split-K chunking may differ); if any member
    does not qualify, every member takes its own path.  Installed by the HF attention wrapper for
    the duration of one forward (plugins/huggingface.py ``_QuantAttention``)."""

    def __init__(self, mods):
        self.mods = list(mods)
        self.tried = False
        self.key = None
        self.outs = {}

    def take(self, mod, input):
        if self.key is not None:
            if input is self.key[0] and input._version == self.key[1]:
                return self.outs.pop(id(mod), None)
            return None
        if self.tried:
            return None
        self.tried = True  # one attempt per forward
        # every member's input quantizer is applied to THIS input up front: only when that has no
        # side effect (a calibrating quantizer would collect a tensor that, for k/v called later
        # with another input -- cross-attention, a device-moving hook -- is not theirs)
        if any(not _input_quantizer_pure(m) for m in self.mods):
            return None
        params = [_fused_params(m, input) for m in self.mods]
        if any(p is None for p in params) or len({p[2][2] for p in params}) != 1:
            return None
        xs = [_fused_input(m, input) for m in self.mods]
        if any(x is None for x in xs):
            # an input quantizer changed the dtype (as in _fused_forward, that member then takes
            # the reference path); the others finish on their own operands
            outs = [None if x is None else self._single(m, x, p) for m, x, p in zip(self.mods, xs, params)]
        else:
            wqs = [m._modules["weight_quantizer"] for m in self.mods]
            kind = params[0][2][2]
            outs = _ops().qlinear_small_m_group(
                xs, [p[0] for p in params], [p[1] for p in params], [p[2][0] for p in params],
                [p[2][1] for p in params], kind, [q._num_bits if kind == 0 else 8 for q in wqs],
                [int(bool(q._unsigned)) for q in wqs], [int(bool(q._narrow_range)) for q in wqs],
            )
        self.key = (input, input._version)
        self.outs = {id(m): y for m, y in zip(self.mods, outs) if m is not mod and y is not None}
        return outs[self.mods.index(mod)]

    @staticmethod
    def _single(m, x, p):
        weight, bias, (amax, block, kind) = p
        wq = m._modules["weight_quantizer"]
        return _ops().qlinear_small_m(x, weight, bias, amax, block, kind, wq._num_bits if kind == 0 else 8,
                                      bool(wq._unsigned), bool(wq._narrow_range))


@QuantModuleRegistry.register({nn.Linear: "nn.Linear"})
class _QuantLinear(QuantLinearConvBase):
    """Quantized base class for nn.Linear type classes: weight per-row INT8 by default."""

    default_quant_desc_weight = tensor_quant.QUANT_DESC_8BIT_LINEAR_WEIGHT_PER_ROW

    def forward(self, input, *args, **kwargs):
        if not args and not kwargs:
            group = self.__dict__.get("_projection_group")
            if group is not None:
                y = group.take(self, input)
                if y is not None:
                    return y
            y = _fused_forward(self, input)
            if y is not None:
                return y
        return super().forward(input, *args, **kwargs)

    @staticmethod
    def quantized_linear_fn(package, func_name, self, input, weight, *args, **kwargs):
        """Quantized version of a generic linear functional (reference :44-53)."""
        output = getattr(package, func_name)(
            self.input_quantizer(input), self.weight_quantizer(weight), *args, **kwargs
        )
        return self.output_quantizer(output)


class QuantLinear(nn.Linear):
    """``nn.Linear`` that is born quantized (legacy constructor form, reference :56-61).  The
    class-level ``default_quant_desc_input`` / ``default_quant_desc_weight`` apply when no
    descriptor is passed (reference tests/unit/torch/quantization/test_quant_linear.py:199-222)."""

    default_quant_desc_input = tensor_quant.QUANT_DESC_8BIT_PER_TENSOR
    default_quant_desc_weight = tensor_quant.QUANT_DESC_8BIT_LINEAR_WEIGHT_PER_ROW

    def __new__(cls, *args, quant_desc_input=None, quant_desc_weight=None, **kwargs):
        m = nn.Linear(*args, **kwargs)
        QuantModuleRegistry.convert(m)
        m.input_quantizer.set_from_attribute_config(
            cls.default_quant_desc_input if quant_desc_input is None else quant_desc_input
        )
        m.weight_quantizer.set_from_attribute_config(
            cls.default_quant_desc_weight if quant_desc_weight is None else quant_desc_weight
        )
        return m


Linear = QuantLinear
