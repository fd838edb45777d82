#!/usr/bin/env python3
"""The skip_zeros > 2^24 histogram call alone (bf16 [8192, 14336], every 97th element zero, 2048
bins, 16 torch.histc threads), for rocprofv3 PMC passes: the count launch (hist_value_kernel
NZ mode), the boundary recount and the chunk fold of each call.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python3 scripts/prof_hist_nz.py [ITERS]"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from modelopt_amd.torch.quantization.calib import histogram as H  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 10
x = torch.randn(8192, 14336, device="cuda", generator=torch.Generator(device="cuda").manual_seed(7)).to(torch.bfloat16)
x.view(-1)[::97] = 0
hmax = torch.tensor([16.0 * 6], device="cuda")
for _ in range(ITERS):
    H._histc_counts(x, hmax, 2048, True, threads=16)
torch.cuda.synchronize()
print("elements", x.numel(), "bytes", x.numel() * 2)
