#!/usr/bin/env python3
"""C5 wall-clock split (Mixtral-8x7B dims, FP8_DEFAULT_CFG, 512 x 512 tokens, batch 16): per-batch
times of the bf16 forward (second pass, after a warm-up) and of the calibration forward inside
mtq.quantize, plus the quantize time before the first batch (conversion, weight amax pass) and after
the last one (amax load, checks).  Shows which part of the PTQ-over-bf16 gap is per batch and which
is one-time.  python scripts/prof_c5_batches.py [layers] [samples]"""
import gc
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from benchmarks import ptq_llama  # noqa: E402

layers = int(sys.argv[1]) if len(sys.argv) > 1 else 32
samples = int(sys.argv[2]) if len(sys.argv) > 2 else 512
import modelopt_amd.torch.quantization as mtq  # noqa: E402

dev = torch.device("cuda")
model = ptq_llama.build_model(layers, dev, "mixtral-8x7b")
model.config._experts_implementation = "eager"
g = torch.Generator(device=dev).manual_seed(1234)
ids = torch.randint(0, 32000, (samples, 512), device=dev, generator=g)
batches = list(ids.split(16))
marks = []


def loop(m, rec=None):
    with torch.no_grad():
        for b in batches:
            m(b)
            if rec is not None:
                torch.cuda.synchronize()
                rec.append(time.perf_counter())


loop(model)
gc.collect()  # as benchmarks/ptq_llama.py: the model build's pending collection outside the timing
torch.cuda.synchronize()
bf = [time.perf_counter()]
loop(model, bf)
bf16_batches = [b - a for a, b in zip(bf[:-1], bf[1:])]
print(f"bf16 forward {bf[-1] - bf[0]:.3f} s", file=sys.stderr, flush=True)


def calib_loop(m):
    torch.cuda.synchronize()
    marks.append(time.perf_counter())
    loop(m, marks)


gc.collect()
torch.cuda.synchronize()
t0 = time.perf_counter()
mtq.quantize(model, mtq.FP8_DEFAULT_CFG, calib_loop)
torch.cuda.synchronize()
t1 = time.perf_counter()
cal_batches = [b - a for a, b in zip(marks[:-1], marks[1:])]
out = {
    "layers": layers, "samples": samples,
    "bf16_forward_s": round(bf[-1] - bf[0], 3),
    "ptq_s": round(t1 - t0, 3),
    "before_first_batch_s": round(marks[0] - t0, 3),
    "calibration_forward_s": round(marks[-1] - marks[0], 3),
    "after_last_batch_s": round(t1 - marks[-1], 3),
    "bf16_batch_ms": [round(x * 1e3, 1) for x in bf16_batches],
    "calib_batch_ms": [round(x * 1e3, 1) for x in cal_batches],
}
print(json.dumps(out))
