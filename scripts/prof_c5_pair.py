#!/usr/bin/env python3
"""C5 calibration-forward overhead against the plain HF model, paired in one process: two
Mixtral-8x7B-dims models resident at once (2 x 93 GB), the plain bf16 one and one converted by
mtq.quantize(FP8_DEFAULT_CFG) and put back into max-collection mode; rounds alternate a pass over
the calibration set through each (plus variants of the converted one), so clock drift and
box-to-box spread cancel.  Variants: `side` = the product (MoE collects on the side stream),
`noside` = the same collects on the main stream.
    python scripts/prof_c5_pair.py [layers] [samples] [rounds]"""
import contextlib
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
from modelopt_amd.torch.quantization.plugins import huggingface as hf  # noqa: E402

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
real_beside = hf._beside


@contextlib.contextmanager
def _main_stream(side, *inputs):
    yield


def timed(m, variant=None):
    if m is quant:
        enable_stats_collection(quant)
        hf._beside = real_beside if variant == "side" else _main_stream
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
res = {"layers": layers, "samples": samples, "plain_s": [], "side_s": [], "noside_s": []}
for _ in range(rounds):
    res["plain_s"].append(round(timed(plain), 4))
    res["side_s"].append(round(timed(quant, "side"), 4))
    res["noside_s"].append(round(timed(quant, "noside"), 4))
hf._beside = real_beside
p = statistics.median(res["plain_s"])
for v in ("side", "noside"):
    res[f"{v}_overhead_median"] = round(statistics.median(res[f"{v}_s"]) / p - 1, 4)
print(json.dumps(res))
