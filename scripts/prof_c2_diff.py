#!/usr/bin/env python3
"""C2 (Llama-3-8B FP8_DEFAULT_CFG) calibration forward vs the bf16 forward, kernel by kernel: the
same 4 batches of 16 x 512 tokens profiled (torch.profiler, device time per kernel name) once
without quantizers and once as mtq.quantize's forward_loop, printed as a diff sorted by the extra
device time, plus host wall per batch of both (device synchronised per batch).
    python scripts/prof_c2_diff.py [batches] [model] [config]   (e.g. 4 mixtral-8x7b FP8_DEFAULT_CFG)"""
import json
import sys
import time
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from scripts import ptq_llama  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
model_name = sys.argv[2] if len(sys.argv) > 2 else "llama3-8b"
config = sys.argv[3] if len(sys.argv) > 3 else "FP8_DEFAULT_CFG"
import modelopt_amd.torch.quantization as mtq  # noqa: E402

dev = torch.device("cuda")
model = ptq_llama.build_model(32, dev, model_name)
if model_name.startswith("mixtral"):
    model.config._experts_implementation = "eager"
vocab = ptq_llama.MODELS[model_name][1]["vocab_size"]
g = torch.Generator(device=dev).manual_seed(1234)
batches = list(torch.randint(0, vocab, (16 * nb, 512), device=dev, generator=g).split(16))


def kernel_table(prof):
    t = defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        if e.device_type == torch.autograd.DeviceType.CUDA:
            t[e.name][0] += 1
            t[e.name][1] += e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
    return t


def run(m, walls):
    with torch.no_grad():
        for b in batches:
            t0 = time.perf_counter()
            m(b)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)


run(model, [])
bf_w = []
with profile(activities=[ProfilerActivity.CUDA]) as p0:
    run(model, bf_w)
cal_w = []
prof = {}


def loop(m):
    with profile(activities=[ProfilerActivity.CUDA]) as p1:
        run(m, cal_w)
    prof["p1"] = p1


mtq.quantize(model, getattr(mtq, config), loop)
a, b = kernel_table(p0), kernel_table(prof["p1"])
rows = []
for k in set(a) | set(b):
    ca, ta = a.get(k, [0, 0.0])
    cb, tb = b.get(k, [0, 0.0])
    rows.append((tb - ta, k[:110], ca, cb, round(ta / 1e3, 2), round(tb / 1e3, 2)))
rows.sort(reverse=True)
print(json.dumps({"bf16_batch_ms": [round(w * 1e3, 1) for w in bf_w], "calib_batch_ms": [round(w * 1e3, 1) for w in cal_w],
                  "bf16_kernel_ms": round(sum(t for _, t in a.values()) / 1e3, 2),
                  "calib_kernel_ms": round(sum(t for _, t in b.values()) / 1e3, 2)}))
for r in rows[:40]:
    print(f"{r[0] / 1e3:9.3f} ms  bf16 {r[2]:6d} {r[4]:9.2f} ms  calib {r[3]:6d} {r[5]:9.2f} ms  {r[1]}")
