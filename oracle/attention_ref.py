"""CPU restatement of the reference's flash attention with softmax-P quant-dequant -- TEST
INFRASTRUCTURE (the oracle for ``mtq_attention_fwd``; see oracle/ref_ops.py for the rules: only
tests/, smoke() and bench.py's cpu_baseline may import it, never the product).

Follows modelopt/torch/kernels/common/attention/triton_fa.py ``_attn_fwd`` (:255-516) per query
row and per 32-key tile (BLOCK_N = 32, the only N of its autotune configs :86-89):

* scores ``(q . k) * qk_scale`` with ``qk_scale = sm_scale * LOG2E`` (:922), masked keys -inf
  (``_apply_mask`` :194-217, causal queries are the last ``len_q`` positions of the key span);
* online softmax (:426-432): ``m' = max(m, rowmax)``, ``p = exp2(s - m')``, ``c = exp2(m - m')``,
  ``l = l c + sum p``, ``acc = acc c``;
* P qdq (:436-451): FP8 ``fp8_scalar_qdq`` (common/fp8_quant.py) with ``S = amax / 448``;
  NVFP4 ``_p_qdq_nvfp4`` (attention/bmm2_qdq.py:37-61 -> common/nvfp4_quant.py:129-155) on p
  rounded to the V dtype, blocks of 16 keys, ``S = amax / (6 * 448)``;
* BMM2 (:486-489): FP8/none ``p.to(v.dtype) @ v`` accumulated in fp32, NVFP4 an fp32 dot;
* ``o = acc / max(l, 1e-6)`` (:495), rows past ``len_q`` not written (left as zero here).

Pinned by tests/golden/attention.* (the reference's own Triton kernel run by the interpreter,
tests/golden/make_golden_attention.py): tests/test_oracle_attention.py.
"""

from __future__ import annotations

import math

import torch

LOG2E = 1.44269504088896
BLOCK_N = 32


def _fp8_rt(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.float8_e4m3fn).float()


def fp8_scalar_qdq(x: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """common/fp8_quant.py fp8_scalar_qdq: ``cast_e4m3(clamp(x / S, +-448)) * S``."""
    return _fp8_rt(torch.clamp(x / scale, -448.0, 448.0)) * scale


def _fp4_round_magnitude(a: torch.Tensor) -> torch.Tensor:
    """common/nvfp4_quant.py fp4_round_magnitude (thresholds, ties to even)."""
    out = torch.full_like(a, 6.0)
    for thr, val, le in ((5.0, 4.0, True), (3.5, 3.0, False), (2.5, 2.0, True), (1.75, 1.5, False),
                         (1.25, 1.0, True), (0.75, 0.5, False), (0.25, 0.0, True)):
        sel = a <= thr if le else a < thr
        out = torch.where(sel, torch.tensor(val), out)
    return out


def nvfp4_p_qdq(p: torch.Tensor, global_scale: torch.Tensor) -> torch.Tensor:
    """bmm2_qdq._p_qdq_nvfp4 on a [rows, 32] fp32 tile: per 16 keys, ``fp8_quantize_scale``
    then ``nvfp4_scalar_quant`` (p >= 0, so the block amax is a plain max)."""
    r, n = p.shape
    g = p.reshape(r, n // 16, 16)
    bmax = g.amax(dim=-1, keepdim=True)
    s8 = torch.minimum(bmax / (torch.tensor(6.0) * global_scale), torch.tensor(448.0))
    scale = _fp8_rt(s8) * global_scale
    zero = scale == 0.0
    safe = torch.where(zero | torch.isnan(scale) | (scale.abs() == math.inf), torch.tensor(1.0), scale)
    q = _fp4_round_magnitude(g.abs() / safe) * safe
    q = torch.where(g >= 0, q, -q)
    return torch.where(zero, torch.tensor(0.0), q).reshape(r, n)


def attention_fwd(q, k, v, b_start_loc, b_seq_len, b_start_loc_k=None, b_seq_len_k=None,
                  is_causal=True, softmax_scale=None, p_qdq=None, p_qdq_amax=1.0):
    """Restated ``attention()`` forward on flat varlen tensors q [Tq, Hq, D], k/v [Tk, Hkv, D]."""
    if b_seq_len_k is None:
        b_start_loc_k, b_seq_len_k = b_start_loc, b_seq_len
    d = q.shape[-1]
    hq, hkv = q.shape[1], k.shape[1]
    grp = hq // hkv
    sm = d ** -0.5 if softmax_scale is None else softmax_scale
    qk_scale = torch.tensor(sm * LOG2E, dtype=torch.float32)  # Python double -> fp32 kernel arg
    if p_qdq == "fp8":
        pscale = torch.tensor(p_qdq_amax / 448.0, dtype=torch.float32)
    elif p_qdq == "nvfp4":
        pscale = torch.tensor(p_qdq_amax / (6.0 * 448.0), dtype=torch.float32)
    o = torch.zeros(q.shape, dtype=q.dtype)
    ninf = torch.tensor(-math.inf)
    for b in range(len(b_seq_len)):
        lq, lk = int(b_seq_len[b]), int(b_seq_len_k[b])
        sq, sk = int(b_start_loc[b]), int(b_start_loc_k[b])
        off = lk - lq
        for h in range(hq):
            kh = h // grp
            qq = q[sq:sq + lq, h].float()
            kk = k[sk:sk + lk, kh]
            vv = v[sk:sk + lk, kh]
            m = torch.full((lq,), -math.inf)
            ell = torch.zeros(lq)
            acc = torch.zeros(lq, d)
            qpos = torch.arange(lq)
            bound = min(off + lq, lk) if is_causal else lk
            for kv0 in range(0, max(bound, 0), BLOCK_N):
                kpos = kv0 + torch.arange(BLOCK_N)
                kt = torch.zeros(BLOCK_N, d, dtype=k.dtype)
                vt = torch.zeros(BLOCK_N, d, dtype=v.dtype)
                nv = max(0, min(BLOCK_N, lk - kv0))
                kt[:nv], vt[:nv] = kk[kv0:kv0 + nv], vv[kv0:kv0 + nv]
                s = (qq @ kt.float().T) * qk_scale
                ok = kpos[None, :] < lk
                if is_causal:
                    ok = ok & (qpos[:, None] + off >= kpos[None, :])
                s = torch.where(ok, s, ninf)
                mn = torch.maximum(m, s.amax(dim=1))
                mu = torch.where(mn == -math.inf, torch.tensor(0.0), mn)
                p = torch.exp2(s - mu[:, None])
                corr = torch.where(m == mn, torch.tensor(1.0), torch.exp2(m - mu))
                ell = ell * corr + p.sum(dim=1)
                acc = acc * corr[:, None]
                if p_qdq == "fp8":
                    p = fp8_scalar_qdq(p, pscale)
                elif p_qdq == "nvfp4":
                    p = nvfp4_p_qdq(p.to(v.dtype).float(), pscale)
                if p_qdq == "nvfp4":
                    acc = acc + p.double().matmul(vt.double()).float()
                else:
                    acc = acc + p.to(v.dtype).double().matmul(vt.double()).float()
                m = mn
            out = acc / torch.clamp(ell, min=1e-6)[:, None]
            o[sq:sq + lq, h] = out.to(q.dtype)
    return o
