#!/usr/bin/env python3
"""C3 (Llama-3-8B INT4_AWQ_CFG) per-batch wall time of both AWQ-lite passes (caching and search),
device synchronised per batch, 6 batches of 16 x 512 tokens: a first batch far above the rest is
host time (first-use kernel loads, allocations), the rest is the steady state."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from scripts import ptq_llama  # noqa: E402

import modelopt_amd.torch.quantization as mtq  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dev = torch.device("cuda")
model = ptq_llama.build_model(32, dev, "llama3-8b")
g = torch.Generator(device=dev).manual_seed(1234)
batches = list(torch.randint(0, 128256, (16 * nb, 512), device=dev, generator=g).split(16))
with torch.no_grad():
    for b in batches[:2]:
        model(b)
torch.cuda.synchronize()
passes = []


def loop(m):
    ts = []
    torch.cuda.synchronize()
    with torch.no_grad():
        for b in batches:
            t0 = time.perf_counter()
            m(b)
            torch.cuda.synchronize()
            ts.append(round((time.perf_counter() - t0) * 1e3, 1))
    passes.append(ts)
    print(f"pass {len(passes)}: batch ms {ts}", flush=True)


t0 = time.perf_counter()
mtq.quantize(model, mtq.INT4_AWQ_CFG, loop)
torch.cuda.synchronize()
print(f"quantize {time.perf_counter() - t0:.2f} s; passes {[round(sum(p) / 1e3, 2) for p in passes]} s", flush=True)
