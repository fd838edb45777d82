#!/usr/bin/env python3
"""Host-side profile of C5 (Mixtral-8x7B dims, FP8_DEFAULT_CFG) at reduced depth: bf16 forward vs
mtq.quantize wall-clock and a cProfile of the quantize call (top functions by own time), to see
where the quantizer overhead on top of the eager expert loop goes.
    python scripts/prof_c5.py [layers] [samples]"""
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from benchmarks import ptq_llama  # noqa: E402

layers = int(sys.argv[1]) if len(sys.argv) > 1 else 4
samples = int(sys.argv[2]) if len(sys.argv) > 2 else 256
profile = "--no-cprofile" not in sys.argv
import modelopt_amd.torch.quantization as mtq  # noqa: E402

dev = torch.device("cuda")
model = ptq_llama.build_model(layers, dev, "mixtral-8x7b")
model.config._experts_implementation = "eager"
ids = torch.randint(0, 32000, (samples, 512), device=dev, generator=torch.Generator(device=dev).manual_seed(1))
batches = list(ids.split(16))


def loop(m):
    with torch.no_grad():
        for b in batches:
            m(b)


calib_s = []


def timed_loop(m):
    torch.cuda.synchronize()
    t = time.perf_counter()
    loop(m)
    torch.cuda.synchronize()
    calib_s.append(time.perf_counter() - t)


loop(model)
torch.cuda.synchronize()
t0 = time.perf_counter()
loop(model)
torch.cuda.synchronize()
bf16 = time.perf_counter() - t0
pr = cProfile.Profile()
torch.cuda.synchronize()
t0 = time.perf_counter()
if profile:
    pr.enable()
mtq.quantize(model, mtq.FP8_DEFAULT_CFG, timed_loop)
torch.cuda.synchronize()
if profile:
    pr.disable()
ptq = time.perf_counter() - t0
t0 = time.perf_counter()
loop(model)
torch.cuda.synchronize()
qfwd = time.perf_counter() - t0
print(f"layers {layers} samples {samples}: bf16 forward {bf16:.3f} s, ptq {ptq:.3f} s (calibration forward "
      f"{calib_s[0]:.3f} s, the rest {ptq - calib_s[0]:.3f} s), fake-quant forward {qfwd:.3f} s", flush=True)
if not profile:
    sys.exit(0)
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
print(s.getvalue())
