#!/usr/bin/env python3
"""Python cyclic-GC time inside the first mtq.quantize of the process (C2: Llama-3-8B
FP8_DEFAULT_CFG, 512 x 512 tokens, bench.py's order): collections per generation and their
total duration, from gc.callbacks.  Prints one JSON line."""
import gc
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402


def main():
    import modelopt_amd.torch.quantization as mtq
    from scripts.ptq_llama import build_model

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = build_model(32, dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    ids = torch.randint(0, 128256, (512, 512), device=dev, generator=g)
    batches = list(ids.split(16))

    def forward_loop(m):
        with torch.no_grad():
            for b in batches:
                m(b)

    forward_loop(model)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    forward_loop(model)
    torch.cuda.synchronize()
    res = {"bf16_forward_s": round(time.perf_counter() - t0, 4), "objects": len(gc.get_objects())}
    stats = {0: [0, 0.0], 1: [0, 0.0], 2: [0, 0.0]}
    start = {}

    def cb(phase, info):
        if phase == "start":
            start["t"] = time.perf_counter()
        else:
            s = stats[info["generation"]]
            s[0] += 1
            s[1] += time.perf_counter() - start["t"]

    gc.callbacks.append(cb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mtq.quantize(model, mtq.FP8_DEFAULT_CFG, forward_loop)
    torch.cuda.synchronize()
    res["ptq_wall_clock_s"] = round(time.perf_counter() - t0, 4)
    gc.callbacks.remove(cb)
    res["gc"] = {f"gen{k}": {"collections": v[0], "s": round(v[1], 4)} for k, v in stats.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
