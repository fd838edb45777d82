#!/usr/bin/env python3
"""r05 A/B of the per-tensor FP8 export kernel forms on the bench.py input (4 rotating bf16
[32768, 4096] buffers, scale 8 / 448): one vector per lane with 8-byte stores (the product kernel)
against two adjacent vectors per lane with one 16-byte store, U = 1 / 2 (a variant since removed;
result: profiles/r05/export/export_fp8_store_width_ab_r05k.log, 0.78-0.79 vs 0.71-0.73).  Prints
ms, the HBM fraction at 3 B / element and a hash of the output.  Copy to scripts/ to run it on the
box (scripts/exp is not uploaded)."""
import hashlib
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from modelopt_amd import _ext  # noqa: E402

ops = _ext.ops()
g = torch.Generator(device="cuda").manual_seed(1234)
xs = [torch.randn(32768, 4096, device="cuda", generator=g).to(torch.bfloat16) for _ in range(4)]
s = torch.tensor([8.0 / 448], device="cuda")
for _ in range(10):
    for x in xs:
        ops.export_fp8(x, s, False, True)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
iters = 80
e0.record()
for i in range(iters):
    ops.export_fp8(xs[i % 4], s, False, True)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
h = hashlib.sha256(ops.export_fp8(xs[0], s, False, True).view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]
n = xs[0].numel()
print(json.dumps({"pt2": os.environ.get("MTQ_EXP_PT2", "0"), "ms": round(ms, 4),
                  "frac": round(n * 3 / (ms * 1e-3) / 8e12, 4), "hash": h}))
