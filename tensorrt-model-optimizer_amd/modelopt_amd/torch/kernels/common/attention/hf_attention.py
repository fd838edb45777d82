"""HuggingFace attention-interface wrapper around the MFMA flash attention (reference
modelopt/torch/kernels/common/attention/hf_triton_attention.py:35-282).

The envelope checks and the varlen metadata are the reference's (same errors for sliding
windows, sinks, softcapping, non-causal masks, left / holed padding, multi-token forwards over a
longer cache).  MI355X-first difference: the reference permutes q/k/v into contiguous
``[B * S, H, D]`` copies; here the kernel reads HF's ``[B, H, S, D]`` states through their strides
(batch / token / head strides, no copies) and writes ``[B, S, H, D]`` directly.
"""

from __future__ import annotations

import torch
import torch.nn as nn

from .flash_attention import attention_into


def _seq_lens_from_mask(attention_mask, fallback: int, device) -> tuple[torch.Tensor | None, bool]:
    """Per-sequence lengths of a right-padded 2D mask (reference :35-50)."""
    if attention_mask is not None and attention_mask.dim() == 2:
        mask = attention_mask.bool() if attention_mask.dtype != torch.bool else attention_mask
        b_seq_len = mask.sum(dim=1).to(torch.int32).to(device)
        return b_seq_len, bool((b_seq_len != fallback).any())
    return None, False


def _check_mask_supported(attention_mask, seq_q: int) -> None:
    """Reject masks the varlen metadata would misread (reference :53-93)."""

    def _unsupported(reason):
        return NotImplementedError(
            f"The ModelOpt Triton attention kernel does not support {reason}. "
            "Use unpadded (or uniform-length) right-padded inputs."
        )

    if attention_mask is None:
        return
    if attention_mask.dim() == 2:
        if attention_mask.shape[1] != seq_q:
            raise _unsupported("padded batches during cached decode")
        mask_bool = attention_mask.to(torch.bool)
        if not mask_bool[:, 0].all():
            raise _unsupported("left-padded inputs")
        if not (mask_bool[:, :-1].int() >= mask_bool[:, 1:].int()).all():
            raise _unsupported("non-contiguously padded inputs")
        return
    last_row = attention_mask[..., -1, :]
    hidden = ~last_row if attention_mask.dtype == torch.bool else last_row != 0
    if hidden.any():
        raise _unsupported("masks carrying padding or non-causal structure")


def validate_attention_envelope(module: nn.Module, query, key, attention_mask, **kwargs) -> None:
    """Raise ``NotImplementedError`` for inputs outside the kernel / wrapper envelope (reference
    ``validate_triton_attention_envelope`` :96-151; the messages are the reference's)."""
    if getattr(module, "sliding_window", None) or kwargs.get("sliding_window"):
        raise NotImplementedError(
            "The ModelOpt Triton attention kernel does not support sliding-window attention layers."
        )
    for name, reason in (("s_aux", "attention sinks"), ("softcap", "logit softcapping")):
        if kwargs.get(name) is not None:
            raise NotImplementedError(
                f"The ModelOpt Triton attention kernel does not support {reason} ('{name}')."
            )
    if kwargs.get("is_causal") is False or getattr(module, "is_causal", True) is False:
        raise NotImplementedError("The ModelOpt Triton attention kernel does not support non-causal attention.")
    if kwargs.get("dropout"):
        raise NotImplementedError(
            "The ModelOpt Triton attention kernel does not support attention dropout; "
            "set attention_dropout=0 for training."
        )
    if query.shape[-1] < 16:
        raise NotImplementedError(
            f"The ModelOpt Triton attention kernel requires head_dim >= 16, got {query.shape[-1]}."
        )
    seq_q, seq_k = query.shape[2], key.shape[2]
    if seq_q > 1 and seq_k != seq_q:
        raise NotImplementedError(
            "The ModelOpt Triton attention kernel does not support multi-token "
            "forwards over a longer KV cache (chunked prefill or "
            "assisted/speculative decoding)."
        )
    _check_mask_supported(attention_mask, seq_q)


def _kernel_view(t: torch.Tensor) -> torch.Tensor:
    """[B, H, S, D] -> a [B, S, H, D] view the kernel can read (16-byte rows); copy only when the
    strides or the base address do not allow it."""
    x = t.transpose(1, 2)
    ec = 16 // x.element_size()
    if x.stride(-1) != 1 or any(s % ec for s in x.stride()[:-1]) or x.data_ptr() % 16:
        x = x.contiguous()
    return x


def attention_forward(
    module: nn.Module,
    query: torch.Tensor,
    key: torch.Tensor,
    value: torch.Tensor,
    attention_mask: torch.Tensor | None,
    scaling: float,
    dropout: float = 0.0,
    p_qdq: str | None = None,
    p_qdq_amax: float | None = None,
    **kwargs,
) -> tuple[torch.Tensor, None]:
    """HF ``AttentionInterface``-compatible forward (reference ``triton_attention_forward``
    :154-281): query ``[B, H, S, D]``, key/value ``[B, H_kv, S_k, D]``; returns
    ``([B, S, H, D], None)``.  Prefill is causal; a single-token query (decode) attends to the
    whole cache.  Padding rows (right-padded 2D mask) are zero."""
    batch, num_heads, seq_len, head_dim = query.shape
    seq_k = key.shape[2]
    device = query.device
    is_decode = seq_len <= 1
    b_seq_len, has_padding = _seq_lens_from_mask(attention_mask, seq_len, device)
    if b_seq_len is None:
        b_seq_len = torch.full((batch,), seq_len, device=device, dtype=torch.int32)
    zeros = torch.zeros(batch, device=device, dtype=torch.int32)
    b_seq_len_k = b_seq_len if not is_decode else torch.full((batch,), seq_k, device=device, dtype=torch.int32)
    q, k, v = _kernel_view(query), _kernel_view(key), _kernel_view(value)
    out = (torch.zeros if has_padding else torch.empty)(batch, seq_len, num_heads, head_dim,
                                                       dtype=query.dtype, device=device)
    attention_into(q, k, v, out, zeros, b_seq_len, seq_len, not is_decode, scaling, zeros, b_seq_len_k,
                   p_qdq, 1.0 if p_qdq_amax is None else p_qdq_amax)
    return out, None


# the reference's names
triton_attention_forward = attention_forward
validate_triton_attention_envelope = validate_attention_envelope
