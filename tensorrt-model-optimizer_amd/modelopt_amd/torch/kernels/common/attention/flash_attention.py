"""Variable-length flash attention with GQA and softmax-P quant-dequant on gfx950 MFMA.

Mirror of the reference's ``attention()`` (modelopt/torch/kernels/common/attention/triton_fa.py:
1221-1390) for the path the quantization plugin takes (plugins/huggingface.py:145-195): same
arguments, same scale conventions (``p_qdq_amax / 448`` for FP8, ``p_qdq_amax / (6 * 448)`` for
NVFP4, default amax 1.0), same error behaviour.  The kernel is ``mtq_attention_fwd``
(csrc/mtq_attention.hip) -- there is no Triton and no fallback: a CPU tensor or a missing
extension raises.

Forward only (calibration / PTQ evaluation): the reference's STE backward, N:M sparse softmax,
skip-softmax, V qdq and the paged KV cache belong to its training / sparse-attention / serving
paths (SURVEY.md §8 out of scope) and raise ``NotImplementedError`` here.
"""

from __future__ import annotations

import math

import torch

from ....._ext import ops

LOG2E: float = 1.44269504088896

_P_QDQ_MODES = {None: 0, "fp8": 1, "nvfp4": 2}
_HEAD_DIMS = (16, 32, 64, 96, 128)


def _p_qdq_scale(p_qdq: str | None, p_qdq_amax: float) -> float:
    """triton_fa.py:1335-1345: the per-tensor amax -> the kernel's scale (a Python double)."""
    if p_qdq is None:
        return 1.0
    if not (math.isfinite(p_qdq_amax) and p_qdq_amax > 0):
        raise ValueError(f"p_qdq_amax must be a finite positive value, got {p_qdq_amax}")
    return p_qdq_amax / 448.0 if p_qdq == "fp8" else p_qdq_amax / (6.0 * 448.0)


def attention_into(q, k, v, out, b_start_loc, b_seq_len, max_input_len, is_causal, sm_scale,
                   b_start_loc_k, b_seq_len_k, p_qdq=None, p_qdq_amax=1.0) -> torch.Tensor:
    """Run the kernel into ``out``.  q/k/v/out: flat ``[tokens, heads, D]`` or strided
    ``[B, S, heads, D]`` views (last dim contiguous); rows past a sequence's length are left
    untouched."""
    if p_qdq not in _P_QDQ_MODES:
        raise ValueError(f"p_qdq must be one of {sorted(k for k in _P_QDQ_MODES if k)} or None, got {p_qdq!r}")
    if q.shape[-1] not in _HEAD_DIMS:
        raise NotImplementedError(f"head_dim {q.shape[-1]} is not supported (supported: {_HEAD_DIMS})")
    if q.dtype not in (torch.bfloat16, torch.float16, torch.float32):
        raise NotImplementedError(f"attention supports bf16 / fp16 / fp32 q/k/v, got {q.dtype}")
    ops().attention_fwd(q, k, v, out, b_start_loc, b_seq_len, b_start_loc_k, b_seq_len_k,
                        int(max_input_len), bool(is_causal), float(sm_scale), _P_QDQ_MODES[p_qdq],
                        _p_qdq_scale(p_qdq, p_qdq_amax))
    return out


def attention(
    q: torch.Tensor,
    k: torch.Tensor,
    v: torch.Tensor,
    b_start_loc: torch.Tensor,
    b_seq_len: torch.Tensor,
    max_input_len: int,
    is_causal: bool = True,
    softmax_scale: float | None = None,
    b_start_loc_k: torch.Tensor | None = None,
    b_seq_len_k: torch.Tensor | None = None,
    max_input_len_k: int | None = None,
    *,
    sparsity_n: int = 0,
    sparsity_m: int = 4,
    dense_sink_tokens: int = 0,
    dense_recent_tokens: int = 64,
    skip_softmax_threshold: float | None = None,
    measure_sparsity: bool = False,
    p_qdq: str | None = None,
    p_qdq_amax: float = 1.0,
    v_qdq: str | None = None,
    v_qdq_amax: float | None = None,
    v_cache_quantized: bool = False,
    k_cache: torch.Tensor | None = None,
    v_cache: torch.Tensor | None = None,
    block_table: torch.Tensor | None = None,
    page_size: int = 16,
) -> torch.Tensor:
    """Flash attention over flat varlen tensors (reference triton_fa.py:1221).

    Args (as the reference): q ``[total_q_tokens, num_q_heads, head_dim]``, k/v
    ``[total_kv_tokens, num_kv_heads, head_dim]``; ``b_start_loc`` / ``b_seq_len`` per-sequence
    query offsets / lengths (``*_k`` for K/V, default = the query ones); ``p_qdq`` ``"fp8"`` or
    ``"nvfp4"`` fake-quantises the softmax probabilities before ``P @ V`` with the per-tensor
    ``p_qdq_amax`` (default 1.0, the bound of the unnormalised P).  Returns ``[total_q_tokens,
    num_q_heads, head_dim]`` (rows past a sequence's length unwritten, as the reference).
    """
    if p_qdq not in _P_QDQ_MODES:
        raise ValueError(f"p_qdq must be one of {sorted(k for k in _P_QDQ_MODES if k)} or None, got {p_qdq!r}")
    if v_qdq not in (None, "nvfp4"):
        raise ValueError(f"v_qdq must be one of ['nvfp4'] or None, got {v_qdq!r}")
    if v_cache_quantized and v_qdq != "nvfp4":
        raise ValueError("v_cache_quantized requires v_qdq='nvfp4'")
    unsupported = {
        "sparsity_n": sparsity_n > 0,
        "skip_softmax_threshold": bool(skip_softmax_threshold),
        "measure_sparsity": measure_sparsity,
        "v_qdq": v_qdq is not None,
        "paged KV cache": k_cache is not None or v_cache is not None or block_table is not None,
    }
    bad = [n for n, on in unsupported.items() if on]
    if bad:
        raise NotImplementedError(f"attention: {', '.join(bad)} are outside the MI355X P-qdq path")
    if torch.is_grad_enabled() and any(t.requires_grad for t in (q, k, v)):
        raise NotImplementedError("attention: forward only (calibration); the STE backward is not implemented")
    if not q.is_cuda:
        raise RuntimeError("attention: q/k/v must be on a ROCm (HIP) device; the MI355X-native path has no CPU kernels")
    if q.shape[1] % k.shape[1] != 0:
        raise ValueError(f"num_q_heads {q.shape[1]} must be a multiple of num_kv_heads {k.shape[1]}")
    if b_seq_len_k is None:
        b_start_loc_k, b_seq_len_k = b_start_loc, b_seq_len
    if b_start_loc_k is None:
        b_start_loc_k = torch.zeros_like(b_start_loc)
    sm_scale = 1.0 / (q.shape[2] ** 0.5) if softmax_scale is None else softmax_scale
    o = torch.empty_like(q)
    return attention_into(q, k, v, o, b_start_loc, b_seq_len, max_input_len, is_causal, sm_scale,
                          b_start_loc_k, b_seq_len_k, p_qdq, p_qdq_amax)
