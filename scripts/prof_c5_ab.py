#!/usr/bin/env python3
"""C5 per-batch quantizer overhead, interleaved in one process (Mixtral-8x7B dims): after one
mtq.quantize(FP8_DEFAULT_CFG), rounds of (a) the calibration forward loop with the quantizers
collecting (max calibration's forward, `enable_stats_collection`) and (b) the same loop with every
quantizer disabled (the module wrappers alone, ~ the bf16 forward), so box-to-box clock drift
cancels.  python scripts/prof_c5_ab.py [layers] [samples] [rounds]"""
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
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
import modelopt_amd.torch.quantization as mtq  # noqa: E402
from modelopt_amd.torch.quantization.model_calib import enable_stats_collection, finish_stats_collection  # noqa: E402

dev = torch.device("cuda")
ids = torch.randint(0, 32000, (samples, 512), device=dev, generator=torch.Generator(device=dev).manual_seed(1))
batches = list(ids.split(16))
model = ptq_llama.build_model(layers, dev, "mixtral-8x7b")
model.config._experts_implementation = "eager"


def loop():
    with torch.no_grad():
        for b in batches:
            model(b)


mtq.quantize(model, mtq.FP8_DEFAULT_CFG, lambda m: loop())
qs = [m for m in model.modules() if isinstance(m, mtq.TensorQuantizer)]
enabled = [q for q in qs if q.is_enabled]


def timed(setup):
    setup()
    torch.cuda.synchronize()
    t = time.perf_counter()
    loop()
    torch.cuda.synchronize()
    return time.perf_counter() - t


def calib_on():
    for q in enabled:
        q.enable()
    enable_stats_collection(model)


def all_off():
    for q in qs:
        q.disable()


res = {"layers": layers, "samples": samples, "calib_s": [], "disabled_s": []}
for _ in range(rounds):
    res["disabled_s"].append(round(timed(all_off), 3))
    res["calib_s"].append(round(timed(calib_on), 3))
    finish_stats_collection(model)
res["overhead"] = round(sum(res["calib_s"]) / sum(res["disabled_s"]) - 1, 4)
print(json.dumps(res))
