#!/usr/bin/env python3
"""Why are the first two calibration batches of C2 (Llama-3-8B FP8_DEFAULT_CFG) ~110 ms slower
than the rest (scripts/prof_c2_diff.py)?  Host profile (cProfile) of calibration batches 1, 2 and
3 inside mtq.quantize's forward_loop, device synchronised per batch; top functions by total time."""
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from scripts import ptq_llama  # noqa: E402

import modelopt_amd.torch.quantization as mtq  # noqa: E402

dev = torch.device("cuda")
model = ptq_llama.build_model(32, dev, "llama3-8b")
g = torch.Generator(device=dev).manual_seed(1234)
batches = list(torch.randint(0, 128256, (16 * 4, 512), device=dev, generator=g).split(16))
with torch.no_grad():
    for b in batches:
        model(b)
torch.cuda.synchronize()


def loop(m):
    with torch.no_grad():
        for i, b in enumerate(batches):
            pr = cProfile.Profile()
            t0 = time.perf_counter()
            pr.enable()
            m(b)
            torch.cuda.synchronize()
            pr.disable()
            print(f"=== calibration batch {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
            if i < 3:
                s = io.StringIO()
                pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
                print(s.getvalue(), flush=True)


mtq.quantize(model, mtq.FP8_DEFAULT_CFG, loop)
