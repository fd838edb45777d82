"""Fake-quant functionals over the MI355X-native ops (reference: tensor_quant.py).

The autograd Functions keep the reference's names, argument order and straight-through-estimator
backward (tensor_quant.py:279-568); their forward calls ``torch.ops.modelopt_amd.*`` (HIP kernels
behind include/mtq_amd.h).  ``quantize_op`` / ``dynamic_block_quantize_op`` carry the reference's
torch.library schemas (tensor_quant.py:222-276) in the ``modelopt_amd`` namespace and, as aliases,
under the reference's own ``tensorrt::`` names.  There is no ATen fallback: a missing extension
raises; CPU tensors run the product's host kernels for INT / FP8 (the reference's "cpu" key)
and raise for the other formats.
"""

from __future__ import annotations

import os

import torch
from torch.autograd import Function

from modelopt_amd._ext import ops as _ops

from .config import QuantizerAttributeConfig

__all__ = [
    "DynamicBlockQuantizationFunction",
    "FakeTensorQuantFunction",
    "ScaledE4M3Function",
    "dynamic_block_quant",
    "dynamic_block_quantize_op",
    "e4m3_cast",
    "fake_tensor_quant",
    "fp8_fake_quant",
    "mx_format_map",
    "quantize_op",
    "scaled_e4m3",
]

mx_format_map = {
    (4, 3): "E4M3",
    (5, 2): "E5M2",
    (3, 2): "E3M2",
    (2, 3): "E2M3",
    8: "INT8",
    (8, 0): "E8M0",
    (2, 1): "E2M1",
    (1, 2): "E1M2",
    (0, 3): "E0M3",
    (3, 0): "E3M0",
}

FORMAT_CODES = {
    "E4M3": 0, "E5M2": 1, "INT8": 2, "E0M3": 3, "E1M2": 4, "E3M0": 5, "E2M1": 6, "E3M2": 7,
    "E2M3": 8, "E8M0": 9,
}


def quantize_op(input, amax, num_bits=8, exponent_bits=0, unsigned=False, narrow_range=True):
    """``tensorrt::quantize_op`` schema (tensor_quant.py:222-226) on the HIP kernels."""
    return _ops().quantize_op(input, amax, num_bits, exponent_bits, unsigned, narrow_range)


# tensor_quant.py:43 -- True routes NVFP4 (E2M1 + E4M3 scales) to fused_amax_convert instead of
# the fp4_fake_quant_block kernel (the reference's Triton kernel; here the HIP nvfp4 kernel)
DISABLE_TRITON_KERNEL = False
_disable_synced = [None]


def dynamic_block_quantize_op(
    input, block_size, amax, num_bits, exponent_bits, scale_num_bits, scale_exponent_bits
):
    """``tensorrt::dynamic_block_quantize_op`` schema (tensor_quant.py:227-231)."""
    ops = _ops()
    if _disable_synced[0] is not DISABLE_TRITON_KERNEL:
        ops.set_disable_triton_kernel(bool(DISABLE_TRITON_KERNEL))
        _disable_synced[0] = DISABLE_TRITON_KERNEL
    return ops.dynamic_block_quantize_op(
        input, block_size, amax, num_bits, exponent_bits, scale_num_bits, scale_exponent_bits
    )


def register_reference_op_names() -> bool:
    """Opt-in (call it, or set ``MTQ_AMD_REGISTER_TENSORRT_OPS=1`` before import): register the
    reference's own op names -- ``tensorrt::quantize_op``,
    ``tensorrt::dynamic_block_quantize_op`` and its ``.overload`` (None amax), schemas of
    tensor_quant.py:222-237 -- on the CUDA (= HIP), CPU and Meta keys, so code that calls
    ``torch.ops.tensorrt.*`` directly (or a torch.export graph holding them) runs on these
    kernels.  The ``.overload`` computes the quantization (the reference's implementation of it
    returns ``torch.empty_like(input)``, tensor_quant.py:240-249, uninitialised memory).  When the
    reference package already defined the namespace in this process, its registration stays and
    nothing is replaced (returns False).  Not done by default: once taken here, a reference
    package imported later in the same process would find its namespace defined, swallow the
    error and silently dispatch to these kernels."""
    global REFERENCE_OP_NAMES_REGISTERED
    if REFERENCE_OP_NAMES_REGISTERED:
        return True
    try:
        lib = torch.library.Library("tensorrt", "FRAGMENT")
        lib.define(
            "quantize_op(Tensor input, Tensor amax, int num_bits, int exponent_bits, "
            "bool unsigned, bool narrow_range) -> Tensor"
        )
        lib.define(
            "dynamic_block_quantize_op(Tensor input, int block_size, Tensor amax, int num_bits, "
            "int exponent_bits, int scale_num_bits, int scale_exponent_bits) -> Tensor"
        )
        lib.define(
            "dynamic_block_quantize_op.overload(Tensor input, int block_size, None amax, int num_bits, "
            "int exponent_bits, int scale_num_bits, int scale_exponent_bits) -> Tensor"
        )
    except RuntimeError:
        return False

    def _q(input, amax, num_bits, exponent_bits, unsigned, narrow_range):
        return quantize_op(input, amax, num_bits, exponent_bits, unsigned, narrow_range)

    def _d(input, block_size, amax, num_bits, exponent_bits, scale_num_bits, scale_exponent_bits):
        return dynamic_block_quantize_op(
            input, block_size, amax, num_bits, exponent_bits, scale_num_bits, scale_exponent_bits
        )

    def _fake(input, *args):
        return torch.empty_like(input)

    for key in ("CUDA", "CPU"):
        lib.impl("quantize_op", _q, key)
        lib.impl("dynamic_block_quantize_op", _d, key)
        lib.impl("dynamic_block_quantize_op.overload", _d, key)
    for name in ("quantize_op", "dynamic_block_quantize_op", "dynamic_block_quantize_op.overload"):
        lib.impl(name, _fake, "Meta")
    _REFERENCE_OP_LIB.append(lib)  # keep the registration alive
    REFERENCE_OP_NAMES_REGISTERED = True
    return True


_REFERENCE_OP_LIB: list = []
REFERENCE_OP_NAMES_REGISTERED = False
if os.environ.get("MTQ_AMD_REGISTER_TENSORRT_OPS", "0") == "1":
    register_reference_op_names()


def e4m3_cast(x):
    """Unscaled e4m3 round trip (``_fp8_eager(x, None)``)."""
    return _ops().e4m3_cast(x)


def fp8_fake_quant(x, amax=None):
    """FP8 e4m3 fake quant with optional amax (``fp8_eager`` semantics)."""
    if amax is None:
        return e4m3_cast(x)
    return quantize_op(x, amax, 8, 4, False, False)


E4M3_MAX = 448.0


def compute_fp4_scales(amax, global_amax=None, quantize_block_scales=True, fp8_max_for_normalization=E4M3_MAX):
    """Per-block NVFP4 scales ``amax / 6`` optionally FP8-quantised against the global amax
    (kernels/quantization/gemm/fp4_kernel.py:217-251): small device ops + one FP8 qdq launch."""
    amax = amax.float()
    scale = amax / 6.0
    if quantize_block_scales:
        if global_amax is None:
            global_amax = amax.amax()  # reduce_amax(axis=None) of a non-negative amax
        global_amax = global_amax.float()
        scale_fp8_quant_amax = global_amax * (E4M3_MAX / fp8_max_for_normalization) / 6.0
        scale = fp8_fake_quant(scale, scale_fp8_quant_amax)  # scaled_e4m3_impl
    return scale


def static_blockwise_fp4_fake_quant(
    x, amax, global_amax=None, quantize_block_scales=True, fp8_max_for_normalization=E4M3_MAX,
    out_dtype=None,
):
    """Static two-level NVFP4 fake quant (fp4_kernel.py:254-316): per-block scales from the
    calibrated per-block ``amax`` (and the global amax), then one HIP element pass."""
    n_blocks = amax.numel()
    if x.numel() % n_blocks != 0:
        raise ValueError(
            f"x.numel() ({x.numel()}) is not divisible by amax.numel() ({n_blocks}); "
            "they must satisfy x.numel() == NUM_FP4_BLOCKS * BLOCK_SIZE."
        )
    scale = compute_fp4_scales(amax, global_amax, quantize_block_scales, fp8_max_for_normalization)
    y = _ops().fp4_block_scale_quant(x, scale.reshape(-1))
    if out_dtype is not None and out_dtype != y.dtype:
        y = y.to(out_dtype)
    return y.view(x.shape)


class StaticBlockwiseFP4FakeQuantFunction(Function):
    """Autograd wrapper (tensor_quant.py:571-604): STE with clipping."""

    @staticmethod
    def forward(ctx, x, amax, global_amax=None, quantize_block_scales=True,
                fp8_max_for_normalization=E4M3_MAX, out_dtype=None, pass_through_bwd=False):
        _save_for_backward_if_needed(ctx, pass_through_bwd, x, amax)
        return static_blockwise_fp4_fake_quant(
            x, amax, global_amax, quantize_block_scales, fp8_max_for_normalization, out_dtype
        )

    @staticmethod
    def backward(ctx, grad_outputs):
        return _fake_quant_backward_function(ctx, grad_outputs, num_args=len(ctx.needs_input_grad))


# Predefined descriptors (tensor_quant.py:279-287)
QUANT_DESC_8BIT_PER_TENSOR = QuantizerAttributeConfig(num_bits=8)
QUANT_DESC_UNSIGNED_8BIT_PER_TENSOR = QuantizerAttributeConfig(num_bits=8, unsigned=True)
QUANT_DESC_8BIT_LINEAR_WEIGHT_PER_ROW = QuantizerAttributeConfig(num_bits=8, axis=(0))


# ---- backward: straight-through estimator with clipping (tensor_quant.py:290-316) ----------------


def _fake_tensor_quant_backward(inputs, amax, grad_outputs):
    if amax is None:
        return grad_outputs
    zero = grad_outputs.new_zeros(1)
    return torch.where(inputs.abs() <= amax, grad_outputs, zero)


def _fake_quant_backward_function(ctx, grad_outputs, num_args=1):
    saved = ctx.saved_tensors
    if len(saved) == 0:
        return (grad_outputs,) + (None,) * (num_args - 1)
    inputs, amax = saved
    return (_fake_tensor_quant_backward(inputs, amax, grad_outputs),) + (None,) * (num_args - 1)


def _save_for_backward_if_needed(ctx, pass_through_bwd, inputs, amax):
    if not pass_through_bwd and amax is not None:
        amax = (
            amax
            if isinstance(amax, torch.Tensor)
            else torch.tensor(amax, device=inputs.device, dtype=inputs.dtype)
        )
        ctx.save_for_backward(inputs, amax)


class FakeTensorQuantFunction(Function):
    """INT-n fake quant (tensor_quant.py:319-399)."""

    @staticmethod
    def forward(
        ctx,
        inputs,
        amax,
        bias=None,
        num_bits=8,
        unsigned=False,
        narrow_range=True,
        trt_high_precision_dtype=None,
        pass_through_bwd=False,
        block_size=None,
        axis=None,
    ):
        if bias is not None:
            inputs = inputs - bias
        _save_for_backward_if_needed(ctx, pass_through_bwd, inputs, amax)
        if not isinstance(amax, torch.Tensor):
            amax = torch.tensor(float(amax), device=inputs.device)
        outputs = quantize_op(inputs, amax, num_bits, 0, unsigned, narrow_range)
        if bias is not None:
            outputs = outputs + bias
        return outputs

    @staticmethod
    def backward(ctx, grad_outputs):
        return _fake_quant_backward_function(ctx, grad_outputs, num_args=10)


class ScaledE4M3Function(Function):
    """FP8 e4m3 fake quant (tensor_quant.py:402-460)."""

    @staticmethod
    def forward(ctx, inputs, amax, bias, E, M, trt_high_precision_dtype=None, pass_through_bwd=False):  # noqa: N803
        if E != 4 or M != 3:
            raise NotImplementedError("Only support E=4 & M=3 for now.")
        if bias is not None:
            inputs = inputs - bias
        _save_for_backward_if_needed(ctx, pass_through_bwd, inputs, amax)
        outputs = fp8_fake_quant(inputs, amax)
        if bias is not None:
            outputs = outputs + bias
        return outputs

    @staticmethod
    def backward(ctx, grad_outputs):
        return _fake_quant_backward_function(ctx, grad_outputs, num_args=7)


def _dynamic_block_quantize_forward(ctx, inputs, block_size, amax, num_bits, scale_bits, *_):
    if isinstance(num_bits, int):
        exponent_bits = 0  # MXINT8
    else:
        assert isinstance(num_bits, tuple) and len(num_bits) == 2
        exponent_bits = num_bits[0]
        num_bits = num_bits[0] + num_bits[1] + 1
    assert isinstance(scale_bits, tuple) and len(scale_bits) == 2
    scale_exponent_bits = scale_bits[0]
    scale_num_bits = scale_bits[0] + scale_bits[1] + 1
    return dynamic_block_quantize_op(
        inputs, block_size, amax, num_bits, exponent_bits, scale_num_bits, scale_exponent_bits
    )


class DynamicBlockQuantizationFunction(Function):
    """Dynamic block (MX) fake quant (tensor_quant.py:497-568)."""

    @staticmethod
    def forward(
        ctx,
        inputs,
        block_size,
        amax,
        bias,
        num_bits,
        scale_bits,
        trt_high_precision_dtype=None,
        onnx_quantizer_type="dynamic",
        pass_through_bwd=True,
    ):
        _save_for_backward_if_needed(ctx, pass_through_bwd, inputs, amax)
        return _dynamic_block_quantize_forward(ctx, inputs, block_size, amax, num_bits, scale_bits)

    @staticmethod
    def backward(ctx, grad_outputs):
        return _fake_quant_backward_function(ctx, grad_outputs, num_args=9)


fake_tensor_quant = FakeTensorQuantFunction.apply
scaled_e4m3 = ScaledE4M3Function.apply
dynamic_block_quant = DynamicBlockQuantizationFunction.apply
