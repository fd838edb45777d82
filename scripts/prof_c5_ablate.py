#!/usr/bin/env python3
"""C5 quantizer-overhead ablation at reduced depth (Mixtral-8x7B dims, FP8_DEFAULT_CFG): the
calibration forward loop timed with all quantizers, with only the weight quantizers, with only
the input quantizers, and with every quantizer disabled (the wrappers alone), beside the bf16 loop.
    python scripts/prof_c5_ablate.py [layers] [samples]"""
import copy
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from benchmarks import ptq_llama  # noqa: E402

layers = int(sys.argv[1]) if len(sys.argv) > 1 else 8
samples = int(sys.argv[2]) if len(sys.argv) > 2 else 512
import modelopt_amd.torch.quantization as mtq  # noqa: E402

dev = torch.device("cuda")
ids = torch.randint(0, 32000, (samples, 512), device=dev, generator=torch.Generator(device=dev).manual_seed(1))
batches = list(ids.split(16))


def loop(m):
    with torch.no_grad():
        for b in batches:
            m(b)


def timed_loop(out):
    def f(m):
        torch.cuda.synchronize()
        t = time.perf_counter()
        loop(m)
        torch.cuda.synchronize()
        out.append(time.perf_counter() - t)
    return f


def variant(extra):
    cfg = copy.deepcopy(mtq.FP8_DEFAULT_CFG)
    cfg["quant_cfg"] = list(cfg["quant_cfg"]) + extra
    return cfg


res = {"layers": layers, "samples": samples}
model = ptq_llama.build_model(layers, dev, "mixtral-8x7b")
model.config._experts_implementation = "eager"
loop(model)
torch.cuda.synchronize()
t = time.perf_counter()
loop(model)
torch.cuda.synchronize()
res["bf16_loop_s"] = round(time.perf_counter() - t, 3)
del model
torch.cuda.empty_cache()
for name, extra in (("all", []), ("weights_only", [{"quantizer_name": "*input_quantizer", "enable": False}]),
                    ("inputs_only", [{"quantizer_name": "*weight_quantizer*", "enable": False}]),
                    ("none_enabled", [{"quantizer_name": "*", "enable": False}])):
    model = ptq_llama.build_model(layers, dev, "mixtral-8x7b")
    model.config._experts_implementation = "eager"
    loop(model)  # warm-up of this instance
    cal = []
    torch.cuda.synchronize()
    t = time.perf_counter()
    mtq.quantize(model, variant(extra), timed_loop(cal))
    torch.cuda.synchronize()
    res[name] = {"ptq_s": round(time.perf_counter() - t, 3), "calib_loop_s": round(cal[0], 3) if cal else None}
    print(name, res[name], flush=True)
    del model
    torch.cuda.empty_cache()
print(json.dumps(res))
