"""Fused flash attention with softmax-P qdq (mtq_attention_fwd) on a Llama-3-8B calibration batch:
B = 16 sequences x 512 tokens, 32 query / 8 KV heads, head_dim 128, bf16, causal.

Timed per mode (none / fp8 / nvfp4) with HIP events on the launch stream over back-to-back
launches, against (a) torch SDPA (no P qdq: the unquantised floor) and (b) the eager restatement
a P quantizer needs without a fused kernel (materialised scores, softmax, P fake quant, P @ V).
MFMA FLOP per launch (causal, the reference kernel's work): 4 * B * Hq * D * sum_q (keys seen).

Usage: python benchmarks/attention.py [--iters 20] [--out file.json]
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]

import torch  # noqa: E402

from modelopt_amd.torch.kernels.common.attention import attention  # noqa: E402
from modelopt_amd.torch.quantization.tensor_quant import fp8_fake_quant  # noqa: E402


def timed(fn, iters):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def measure(iters=20, batch=16, seq=512):
    dev = torch.device("cuda")
    B, S, HQ, HKV, D = batch, seq, 32, 8, 128
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B * S, HQ, D, device=dev, generator=g).bfloat16()
    k = torch.randn(B * S, HKV, D, device=dev, generator=g).bfloat16()
    v = torch.randn(B * S, HKV, D, device=dev, generator=g).bfloat16()
    start = (torch.arange(B, device=dev) * S).int()
    lens = torch.full((B,), S, device=dev, dtype=torch.int32)
    flop = 4.0 * B * HQ * D * (S * (S + 1) / 2)  # QK^T + PV over the causal keys
    res = {"shape": {"batch": B, "seq": S, "hq": HQ, "hkv": HKV, "d": D, "dtype": "bf16", "causal": True},
           "flop_per_launch": flop, "peak_tflops_bf16_dense": 2500.0, "modes": {}}
    for mode in (None, "fp8", "nvfp4"):
        ms = timed(lambda: attention(q, k, v, start, lens, S, p_qdq=mode), iters)
        res["modes"][str(mode)] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1)}
    # torch SDPA, no P qdq (HF's default attention)
    qs = q.view(B, S, HQ, D).transpose(1, 2)
    ks = k.view(B, S, HKV, D).transpose(1, 2).repeat_interleave(HQ // HKV, dim=1)
    vs = v.view(B, S, HKV, D).transpose(1, 2).repeat_interleave(HQ // HKV, dim=1)
    ms = timed(lambda: torch.nn.functional.scaled_dot_product_attention(qs, ks, vs, is_causal=True), iters)
    res["sdpa_no_qdq"] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1)}
    # the unfused eager path a P quantizer otherwise needs (scores materialised)
    amax = torch.tensor(1.0, device=dev)
    mask = torch.full((S, S), float("-inf"), device=dev).triu(1)

    def eager():
        s = torch.matmul(qs, ks.transpose(2, 3)) * D ** -0.5 + mask
        p = torch.softmax(s, dim=-1, dtype=torch.float32).to(qs.dtype)
        return torch.matmul(fp8_fake_quant(p, amax), vs)

    ms = timed(eager, max(3, iters // 4))
    res["eager_fp8_p"] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    res = measure(args.iters, args.batch, args.seq)
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
