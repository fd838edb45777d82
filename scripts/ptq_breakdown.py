#!/usr/bin/env python3
"""Where does the PTQ wall-clock go?  Llama-3-8B FP8_DEFAULT_CFG, phase by phase.

Times (host clock, device synchronised at each boundary): convert_to_quantized_model,
enable_stats_collection + weight_only_quantize, the forward_loop with quantizers collecting,
finish_stats_collection (compute_amax / load_calib_amax), promotion + validation, and the same
forward_loop without quantizers.  Also counts quantizer forward calls during calibration.

    python scripts/ptq_breakdown.py [--layers 32] [--samples 512] [--batch 16]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
for p in (str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--samples", type=int, default=512)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--config", default="FP8_DEFAULT_CFG")
    ap.add_argument("--trace", default=None, help="write a torch.profiler chrome trace of one fake-quant batch")
    ap.add_argument("--calib-trace", action="store_true", help="print kernel totals of two calibration batches")
    ap.add_argument("--cold", action="store_true", help="cProfile the first mtq.quantize of the process")
    a = ap.parse_args()

    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization import model_calib as MC
    from modelopt_amd.torch.quantization.config import QuantizeConfig
    from modelopt_amd.torch.quantization.conversion import convert_to_quantized_model
    from modelopt_amd.torch.quantization.nn.modules.tensor_quantizer import TensorQuantizer
    from benchmarks.ptq_llama import build_model

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = build_model(a.layers, dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    ids = torch.randint(0, 128256, (a.samples, a.seq), device=dev, generator=g)
    batches = list(ids.split(a.batch))

    def forward_loop(m):
        with torch.no_grad():
            for b in batches:
                m(b)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, r

    res = {}
    if a.cold:
        # bench.py's order: bf16 warm-up forward, then the first mtq.quantize of the process
        import cProfile
        import io
        import pstats

        forward_loop(model)
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        res["cold_mtq_quantize_s"], _ = timed(lambda: mtq.quantize(model, getattr(mtq, a.config), forward_loop))
        pr.disable()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(45)
        print(buf.getvalue(), file=sys.stderr)
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(30)
        print(buf.getvalue(), file=sys.stderr)
        print(json.dumps(res), flush=True)
        return
    forward_loop(model)
    res["bf16_forward_s"], _ = timed(lambda: forward_loop(model))
    # one forward batch, host-side only (no sync): how long does Python take to enqueue it?
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.no_grad():
        model(batches[0])
    res["bf16_enqueue_one_batch_s"] = time.perf_counter() - t0
    torch.cuda.synchronize()

    cfg = QuantizeConfig(**getattr(mtq, a.config))
    import cProfile
    import io
    import pstats

    pr = cProfile.Profile()
    pr.enable()
    res["convert_s"], _ = timed(lambda: convert_to_quantized_model(model, cfg))
    pr.disable()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(25)
    print(buf.getvalue(), file=sys.stderr)
    res["enable_stats_s"], _ = timed(lambda: (MC.enable_stats_collection(model), MC.weight_only_quantize(model)))

    calls = [0]
    orig = TensorQuantizer.forward

    def counting(self, x):
        calls[0] += 1
        return orig(self, x)

    TensorQuantizer.forward = counting
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            model(batches[0])
        res["calib_enqueue_one_batch_s"] = time.perf_counter() - t0
        torch.cuda.synchronize()
        res["calib_forward_s"], _ = timed(lambda: forward_loop(model))
        if a.calib_trace:
            from torch.profiler import ProfilerActivity, profile

            with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
                with torch.no_grad():
                    for b in batches[:2]:
                        model(b)
                torch.cuda.synchronize()
            print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=30), file=sys.stderr)
    finally:
        TensorQuantizer.forward = orig
    res["quantizer_calls"] = calls[0]
    res["finish_stats_s"], _ = timed(lambda: MC.finish_stats_collection(model))
    res["promote_s"], _ = timed(lambda: MC.promote_static_block_weight_quantizers(model))
    from modelopt_amd.torch.quantization.model_quant import _validate_quantizer_attrs

    res["validate_attrs_s"], _ = timed(lambda: _validate_quantizer_attrs(model))
    if a.trace:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            with torch.no_grad():
                model(batches[0])
            torch.cuda.synchronize()
        prof.export_chrome_trace(a.trace)
        print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25), file=sys.stderr)
    # the real entry point on a fresh model, end to end
    del model
    torch.cuda.empty_cache()
    model = build_model(a.layers, dev)
    res["mtq_quantize_s"], _ = timed(lambda: mtq.quantize(model, getattr(mtq, a.config), forward_loop))
    print(json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
