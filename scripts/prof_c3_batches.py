#!/usr/bin/env python3
"""C3 (Llama-3-8B INT4_AWQ_CFG, 512 x 512 tokens, batch 16) with a synchronised clock after every
batch: the per-batch times of the two awq_lite passes (act-scale caching, search) and the host
phases around them (before the first pass, between the passes, after the last).  The per-batch
syncs cost a little wall-clock; this is a diagnostic, not the bench.
    python scripts/prof_c3_batches.py [layers]"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

import modelopt_amd.torch.quantization as mtq  # noqa: E402
from benchmarks.ptq_llama import build_model  # noqa: E402

layers = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dev = torch.device("cuda")
model = build_model(layers, dev)
g = torch.Generator(device=dev).manual_seed(1234)
ids = torch.randint(0, 128256, (512, 512), device=dev, generator=g)
batches = list(ids.split(16))
with torch.no_grad():
    model(batches[0])
torch.cuda.synchronize()
passes = []


def loop(m):
    times = []
    t = time.perf_counter()
    with torch.no_grad():
        for b in batches:
            m(b)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            times.append(round(t2 - t, 4))
            t = t2
    passes.append((time.perf_counter(), times))


t0 = time.perf_counter()
mtq.quantize(model, mtq.INT4_AWQ_CFG, loop)
torch.cuda.synchronize()
t1 = time.perf_counter()
out = {"layers": layers, "wall_s": round(t1 - t0, 3)}
for i, (tend, times) in enumerate(passes):
    out[f"pass{i}"] = {"sum_s": round(sum(times), 3), "first3": times[:3], "median": sorted(times)[len(times) // 2],
                       "last": times[-1]}
if len(passes) == 2:
    out["before_first_pass_s"] = round(passes[0][0] - sum(passes[0][1]) - t0, 3)
    out["between_passes_s"] = round(passes[1][0] - sum(passes[1][1]) - passes[0][0], 3)
    out["after_last_pass_s"] = round(t1 - passes[1][0], 3)
print(json.dumps(out))
