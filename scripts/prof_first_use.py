#!/usr/bin/env python3
"""First-use cost of the torch kernels the calibration bookkeeping touches (fp32 maximum, zeros,
isnan / isinf / isfinite / any, comparisons, cat) vs their second use, in a fresh process after
one bf16 matmul (the forward's kernels loaded).  Host time per call, device synchronised."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

dev = torch.device("cuda")
a = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
(a @ a).sum().item()
torch.cuda.synchronize()
acc = torch.ones(1, device=dev)
tmp = torch.ones(1, device=dev)
flat = torch.rand(1000, device=dev)
cases = [
    ("torch.zeros fp32", lambda: torch.zeros(1, device=dev)),
    ("tensor.zero_ fp32", lambda: tmp.zero_()),
    ("torch.maximum out=", lambda: torch.maximum(acc, tmp, out=acc)),
    ("torch.cat fp32", lambda: torch.cat([acc, tmp, flat])),
    ("isnan.any", lambda: torch.isnan(flat).any()),
    ("isinf.any", lambda: torch.isinf(flat).any()),
    ("(x<0)|~isfinite .any", lambda: ((flat < 0) | ~torch.isfinite(flat)).any()),
    ("stack.tolist", lambda: torch.stack([flat.any(), flat.any()]).tolist()),
    ("fp32 -> bf16", lambda: flat.to(torch.bfloat16)),
    ("clone fp32", lambda: flat.clone()),
]
from modelopt_amd import _ext  # noqa: E402

ops = _ext.ops()
x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
out = torch.zeros(1, device=dev)
cases.insert(0, ("modelopt_amd amax_accumulate", lambda: ops.amax_accumulate(x, out, 1, 1, x.numel())))
for name, f in cases:
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"{name:32s} first {ts[0]:8.2f} ms, then {ts[1]:.3f} / {ts[2]:.3f} ms", flush=True)
