#!/usr/bin/env python3
"""Driver for rocprofv3 passes on the fused attention kernel (the bench shape: 16 x 512 tokens,
32 / 8 heads, D 128, bf16, causal): a few launches of one P mode.
    python scripts/prof_attn.py [none|fp8|nvfp4] [launches]"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from modelopt_amd.torch.kernels.common.attention import attention  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "fp8"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda")
B, S, HQ, HKV, D = 16, 512, 32, 8, 128
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B * S, HQ, D, device=dev, generator=g).bfloat16()
k = torch.randn(B * S, HKV, D, device=dev, generator=g).bfloat16()
v = torch.randn(B * S, HKV, D, device=dev, generator=g).bfloat16()
start = (torch.arange(B, device=dev) * S).int()
lens = torch.full((B,), S, device=dev, dtype=torch.int32)
for _ in range(n):
    o = attention(q, k, v, start, lens, S, p_qdq=None if mode == "none" else mode)
torch.cuda.synchronize()
print("done", mode, float(o.float().abs().mean()))
