#!/usr/bin/env python3
"""The first AWQ-lite search batch of C3 vs the second under torch.profiler (host ops by self CPU
time): what the ~0.9 s one-time cost of the first search batch is.  3 batches of 16 x 512."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from scripts import ptq_llama  # noqa: E402

import modelopt_amd.torch.quantization as mtq  # noqa: E402

dev = torch.device("cuda")
model = ptq_llama.build_model(32, dev, "llama3-8b")
g = torch.Generator(device=dev).manual_seed(1234)
batches = list(torch.randint(0, 128256, (16 * 3, 512), device=dev, generator=g).split(16))
with torch.no_grad():
    model(batches[0])
torch.cuda.synchronize()
npass = [0]


def loop(m):
    npass[0] += 1
    with torch.no_grad():
        for i, b in enumerate(batches):
            if npass[0] == 2 and i < 2:
                with profile(activities=[ProfilerActivity.CPU]) as p:
                    t0 = time.perf_counter()
                    m(b)
                    torch.cuda.synchronize()
                print(f"=== search batch {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
                print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=25), flush=True)
            else:
                m(b)
        torch.cuda.synchronize()


mtq.quantize(model, mtq.INT4_AWQ_CFG, loop)
