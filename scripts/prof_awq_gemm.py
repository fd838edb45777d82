#!/usr/bin/env python3
"""Driver for rocprofv3 PMC passes on the AWQ search GEMM (gate_proj shape, 11 alphas, M tokens)."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from modelopt_amd import _ext  # noqa: E402

ops = _ext.ops()
dev = torch.device("cuda")
M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
N, K = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (14336, 4096)
G = 11
gen = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(M, K, device=dev, generator=gen).to(torch.bfloat16)
w = (torch.randn(N, K, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
s = torch.rand(G, K, device=dev, generator=gen) * 3 + 0.25
wq = ops.block_quant_dynamic_multi(w, s.to(torch.bfloat16), 128, 4, False, False)
yref = F.linear(x, w)
loss = torch.zeros(G, device=dev)
for _ in range(3):
    ops.awq_search_gemm(x, (1 / s).to(torch.bfloat16), wq, None, yref, loss)
torch.cuda.synchronize()
print("done", loss[:2].tolist())
