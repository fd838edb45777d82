#!/usr/bin/env python3
"""The first replace_quant_module of a process on a Llama-3-8B model resident on the GPU (after a
bf16 forward, bench.py's order), cProfiled, beside a second one on a fresh model: where the
one-time ~0.17 s of the C2 conversion goes."""
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402


def main():
    import modelopt_amd.torch.quantization  # noqa: F401
    from modelopt_amd.torch.quantization.conversion import replace_quant_module
    from scripts.ptq_llama import build_model

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = build_model(32, dev)
    with torch.no_grad():
        model(torch.randint(0, 1000, (2, 64), device=dev))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    t0 = time.perf_counter()
    replace_quant_module(model)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    pr.disable()
    m2 = build_model(2, dev)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    replace_quant_module(m2)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(f"first (32 layers, profiled) {t1 - t0:.4f} s; second (2 layers) {t3 - t2:.4f} s", flush=True)
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(25)
    print(buf.getvalue())
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(40)
    print(buf.getvalue())


if __name__ == "__main__":
    main()
