#!/usr/bin/env python3
"""Driver for rocprofv3 passes on the 11 hipBLASLt GEMMs of one AWQ search batch (the baseline the
search kernel is compared with): x [M, K] @ wq[g]^T for g < 11, gate_proj shape by default."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

dev = torch.device("cuda")
M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
N, K = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (14336, 4096)
gen = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(M, K, device=dev, generator=gen).to(torch.bfloat16)
wq = (torch.randn(11, N, K, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
for _ in range(3):
    for g in range(11):
        F.linear(x, wq[g])
torch.cuda.synchronize()
print("done")
