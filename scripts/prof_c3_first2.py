#!/usr/bin/env python3
"""Follow-up of prof_c3_first.py: where the first AWQ-lite search batch's extra ~0.9 s goes.
Host time (device synchronised around each call) of the per-linear one-time steps of the search
(model_calib._awq_search_tables, _awq_wq_all) and of the fast search call, first search batch vs
the second, 3 batches of 16 x 512 tokens."""
import sys
import time
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from scripts import ptq_llama  # noqa: E402

import modelopt_amd.torch.quantization as mtq  # noqa: E402
from modelopt_amd.torch.quantization import model_calib as MC  # noqa: E402

dev = torch.device("cuda")
model = ptq_llama.build_model(32, dev, "llama3-8b")
g = torch.Generator(device=dev).manual_seed(1234)
batches = list(torch.randint(0, 128256, (16 * 3, 512), device=dev, generator=g).split(16))
with torch.no_grad():
    model(batches[0])
torch.cuda.synchronize()
acc = defaultdict(lambda: [0, 0.0])
first = {}


def wrap(name):
    real = getattr(MC, name)

    def f(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = real(*a, **k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        acc[name][0] += 1
        acc[name][1] += dt
        first.setdefault(name, dt)
        return r

    setattr(MC, name, f)


for n in ("_awq_search_tables", "_awq_wq_all", "_awq_search_fast", "get_scale"):
    wrap(n)
npass = [0]


def loop(m):
    npass[0] += 1
    with torch.no_grad():
        for i, b in enumerate(batches):
            acc.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m(b)
            torch.cuda.synchronize()
            print(f"pass {npass[0]} batch {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms  "
                  + "  ".join(f"{k} n={v[0]} {v[1] * 1e3:.1f} ms" for k, v in acc.items()), flush=True)


mtq.quantize(model, mtq.INT4_AWQ_CFG, loop)
print("first calls (ms):", {k: round(v * 1e3, 2) for k, v in first.items()})
