#!/usr/bin/env python3
"""Goldens for the fused flash attention with softmax-P quant-dequant, from the REFERENCE's own
Triton kernel (modelopt/torch/kernels/common/attention/triton_fa.py ``attention``, ``_attn_fwd``
:255-516; P qdq at :436-451 via kernels/quantization/attention/bmm2_qdq.py and
kernels/quantization/common/{fp8,nvfp4}_quant.py) run on the CPU by the Triton interpreter
(TRITON_INTERPRET=1; same import shims as make_golden.py; run in the survey container only):

    python tests/golden/make_golden_attention.py

Interpreter casts.  Triton 3.6's interpreter narrows fp32 -> bf16 by truncation and fp32 ->
float8e4nv by a mantissa shift that drops carries into the next binade and flushes small values
(see make_golden.gen_nvfp4).  The kernel casts P through both (``p.to(V.dtype)`` before BMM2,
the FP8 P qdq, the NVFP4 block scale), so this script replaces the interpreter's narrowing
helper (``triton.runtime.interpreter._convert_float``) with torch's round-to-nearest-even casts
for fp32 -> {bf16, fp16, float8e4nv} -- what the hardware's ``cvt.rn(.satfinite)`` computes.
Its ``tl.dot`` also multiplies bf16
operands as their raw uint16 bit patterns; they are widened to fp32 (exact) before the matmul.
``libdevice.isnan`` (CUDA's device library, which
the interpreter cannot run) is bound to ``x != x`` in the NVFP4 helper's namespace.  The
reference's source is not modified.  The interpreter's fp32 division and exp2 are numpy's
(IEEE), which the HIP kernel's correctly rounded division matches; its exp2 is v_exp_f32 (1 ulp).

Cases: batch / heads / GQA / head_dim / causal prefill with right padding / decode, bf16 and
fp16, P qdq None, "fp8" (default amax 1 and a calibrated amax) and "nvfp4".
Outputs: attention.safetensors / attention.json.
"""

from __future__ import annotations

import contextlib
import json

import make_golden as mg  # noqa: F401  (installs the import shims, selects the interpreter)
import numpy as np
import torch
from make_golden import OUT, save_file

import triton.runtime.interpreter as _interp

_orig_convert = _interp._convert_float
_NARROW = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp8e4nv": torch.float8_e4m3fn}


def _convert_float_rne(input, input_dtype, output_dtype, rounding_mode):
    name = getattr(output_dtype, "name", None)
    if getattr(input_dtype, "name", None) == "fp32" and name in _NARROW:
        x = torch.from_numpy(np.ascontiguousarray(input).view(np.float32).copy())
        y = x.to(_NARROW[name])
        u = {1: torch.uint8, 2: torch.int16}[y.element_size()]
        out = y.view(u).numpy()
        return out.view(np.uint8 if y.element_size() == 1 else np.uint16)
    return _orig_convert(input, input_dtype, output_dtype, rounding_mode)


_interp._convert_float = _convert_float_rne
_orig_dot = _interp.InterpreterBuilder.create_dot


def _create_dot_bf16(self, a, b, d, input_precision, max_num_imprecise_acc):
    # the interpreter keeps bf16 as raw uint16 and would matmul the bit patterns: widen bf16
    # operands to fp32 first (exact), as the hardware MMA does before its fp32 accumulation
    import triton.language as tl

    def widen(x):
        if x.dtype.scalar == tl.bfloat16:
            return _interp.TensorHandle(
                _orig_convert(x.data, tl.bfloat16, tl.float32, None).view(np.float32), tl.float32)
        return x

    return _orig_dot(self, widen(a), widen(b), d, input_precision, max_num_imprecise_acc)


_interp.InterpreterBuilder.create_dot = _create_dot_bf16
torch.cuda.device = lambda d: contextlib.nullcontext()  # the wrapper's device context, CPU tensors
# no benchmarking driver on the CPU: the autotuner takes its first config (BLOCK_M 16, BLOCK_N 32);
# BLOCK_M only groups query rows (every row's online softmax runs over the same 32-key tiles)
import triton.runtime.autotuner as _at  # noqa: E402

_at.Autotuner._bench = lambda self, *a, config=None, **k: [0.0, 0.0, 0.0]

import modelopt.torch.kernels.quantization.common.nvfp4_quant as _nvq  # noqa: E402
import triton  # noqa: E402
import triton.language as tl  # noqa: E402,F401  (visible to the jit helper below)


@triton.jit
def _isnan(x):
    return x != x


class _InterpLibdevice:
    """``libdevice.isnan`` is a CUDA device-library call the interpreter cannot execute; the
    NVFP4 helper's only use of it (nvfp4_scalar_quant's NaN-scale guard) gets its IEEE meaning."""

    isnan = _isnan


_nvq.libdevice = _InterpLibdevice

from modelopt.torch.kernels.common.attention.triton_fa import attention  # noqa: E402

CASES = [
    # name, dtype, batch, Hq, Hkv, D, lens_q, lens_k (None = same as q), causal, p_qdq, amax
    ("bf16_d64_none", torch.bfloat16, 2, 4, 2, 64, [40, 40], None, True, None, None),
    ("bf16_d64_fp8", torch.bfloat16, 2, 4, 2, 64, [40, 40], None, True, "fp8", None),
    ("bf16_d128_fp8_pad", torch.bfloat16, 2, 4, 1, 128, [70, 33], None, True, "fp8", None),
    ("f16_d64_fp8_amax", torch.float16, 1, 2, 2, 64, [96], None, True, "fp8", 0.6),
    ("bf16_d64_nvfp4", torch.bfloat16, 2, 4, 2, 64, [45, 45], None, True, "nvfp4", None),
    ("f16_d128_nvfp4_pad", torch.float16, 2, 2, 1, 128, [64, 50], None, True, "nvfp4", None),
    ("bf16_d32_nvfp4_amax", torch.bfloat16, 1, 4, 4, 32, [33], None, True, "nvfp4", 0.75),
    ("bf16_d64_decode_fp8", torch.bfloat16, 2, 4, 2, 64, [1, 1], [37, 37], False, "fp8", None),
    ("bf16_d64_decode_nvfp4", torch.bfloat16, 2, 4, 2, 64, [1, 1], [50, 50], False, "nvfp4", None),
]


def main():
    g = torch.Generator().manual_seed(91)
    t, meta = {}, {}
    for name, dt, b, hq, hkv, d, lq, lk, causal, pq, amax in CASES:
        lk = lk or lq
        sq, sk = max(lq), max(lk)
        # flat varlen layout of the reference API: sequence i occupies rows [i * s, i * s + len_i)
        q = (torch.randn(b * sq, hq, d, generator=g) * 1.5).to(dt)
        k = (torch.randn(b * sk, hkv, d, generator=g) * 1.5).to(dt)
        v = torch.randn(b * sk, hkv, d, generator=g).to(dt)
        kw = dict(
            b_start_loc=torch.arange(b, dtype=torch.int32) * sq,
            b_seq_len=torch.tensor(lq, dtype=torch.int32),
            max_input_len=sq,
            is_causal=causal,
            softmax_scale=d ** -0.5,
        )
        if lk is not lq or not causal:
            kw.update(b_start_loc_k=torch.arange(b, dtype=torch.int32) * sk,
                      b_seq_len_k=torch.tensor(lk, dtype=torch.int32), max_input_len_k=sk)
        if pq is not None:
            kw["p_qdq"] = pq
            if amax is not None:
                kw["p_qdq_amax"] = amax
        o = attention(q, k, v, **kw)
        # rows past a sequence's length are never written by the kernel (torch.empty output)
        valid = torch.zeros(b * sq, dtype=torch.bool)
        for i, n in enumerate(lq):
            valid[i * sq: i * sq + n] = True
        o = torch.where(valid[:, None, None], o, torch.zeros((), dtype=o.dtype))
        t[f"{name}.q"], t[f"{name}.k"], t[f"{name}.v"], t[f"{name}.o"] = q, k, v, o
        meta[name] = {"dtype": str(dt).split(".")[-1], "batch": b, "hq": hq, "hkv": hkv, "d": d,
                      "lens_q": lq, "lens_k": lk, "causal": causal, "p_qdq": pq, "amax": amax}
        print(name, tuple(o.shape), float(o.float().abs().max()), flush=True)
    save_file(t, str(OUT / "attention.safetensors"))
    (OUT / "attention.json").write_text(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
