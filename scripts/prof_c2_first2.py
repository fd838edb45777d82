#!/usr/bin/env python3
"""Follow-up of prof_c2_first.py: per-call host time of every amax collect (core_utils.
reduce_amax_accumulate) and every torch.maximum of the first three calibration batches of C2,
once as issued (no sync) and, for batch 0, with the device synchronised before each call."""
import statistics
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from scripts import ptq_llama  # noqa: E402

import modelopt_amd.torch.quantization as mtq  # noqa: E402
from modelopt_amd.torch.quantization.utils import core_utils  # noqa: E402

SYNC = len(sys.argv) > 1 and sys.argv[1] == "sync"
dev = torch.device("cuda")
model = ptq_llama.build_model(32, dev, "llama3-8b")
g = torch.Generator(device=dev).manual_seed(1234)
batches = list(torch.randint(0, 128256, (16 * 4, 512), device=dev, generator=g).split(16))
with torch.no_grad():
    for b in batches:
        model(b)
torch.cuda.synchronize()
rec = {"amax": [], "max": []}
real_acc = core_utils.reduce_amax_accumulate
real_max = torch.maximum


def timed_acc(*a, **k):
    if SYNC:
        torch.cuda.synchronize()
    t = time.perf_counter()
    r = real_acc(*a, **k)
    rec["amax"].append((time.perf_counter() - t) * 1e3)
    return r


def timed_max(*a, **k):
    if SYNC:
        torch.cuda.synchronize()
    t = time.perf_counter()
    r = real_max(*a, **k)
    rec["max"].append((time.perf_counter() - t) * 1e3)
    return r


core_utils.reduce_amax_accumulate = timed_acc
torch.maximum = timed_max


def summary(v):
    if not v:
        return "none"
    s = sorted(v)
    return f"n={len(v)} sum={sum(v):.1f} ms median={statistics.median(v):.3f} max={s[-1]:.2f} top5={[round(x, 2) for x in s[-5:]]} first5={[round(x, 3) for x in v[:5]]}"


def loop(m):
    with torch.no_grad():
        for i, b in enumerate(batches):
            rec["amax"].clear()
            rec["max"].clear()
            t0 = time.perf_counter()
            m(b)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            print(f"batch {i} ({'sync' if SYNC else 'async'}): issue {(t1 - t0) * 1e3:.1f} ms, wall {(time.perf_counter() - t0) * 1e3:.1f} ms")
            print("  amax collects:", summary(rec["amax"]))
            print("  torch.maximum:", summary(rec["max"]), flush=True)


mtq.quantize(model, mtq.FP8_DEFAULT_CFG, loop)
