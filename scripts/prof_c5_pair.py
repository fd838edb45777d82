#!/usr/bin/env python3
"""C5 calibration-forward overhead against the plain HF model, paired in one process: two
Mixtral-8x7B-dims models resident at once (2 x 93 GB), the plain bf16 one and one converted by
mtq.quantize(FP8_DEFAULT_CFG) and put back into max-collection mode; rounds alternate a pass over
the calibration set through each, so clock drift and box-to-box spread cancel.  (r05h measured a
variant with the MoE collects on a side stream here: 4.3 % against 3.0 % on the main stream,
profiles/r05/ptq/c5_pair_side_vs_main_r05h.json; the product keeps them on the main stream.)
    python scripts/prof_c5_pair.py [layers] [samples] [rounds]"""
import gc
import json
import statistics
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
plain = ptq_llama.build_model(layers, dev, "mixtral-8x7b")
plain.config._experts_implementation = "eager"
quant = ptq_llama.build_model(layers, dev, "mixtral-8x7b")
quant.config._experts_implementation = "eager"


def loop(m):
    with torch.no_grad():
        for b in batches:
            m(b)


mtq.quantize(quant, mtq.FP8_DEFAULT_CFG, loop)


def timed(m):
    if m is quant:
        enable_stats_collection(quant)
    gc.collect()
    torch.cuda.synchronize()
    t = time.perf_counter()
    loop(m)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    if m is quant:
        finish_stats_collection(quant)
    return el


loop(plain)  # warm-up
res = {"layers": layers, "samples": samples, "plain_s": [], "calib_s": []}
for _ in range(rounds):
    res["plain_s"].append(round(timed(plain), 4))
    res["calib_s"].append(round(timed(quant), 4))
res["calib_overhead_median"] = round(statistics.median(res["calib_s"]) / statistics.median(res["plain_s"]) - 1, 4)
print(json.dumps(res))
