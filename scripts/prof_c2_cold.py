#!/usr/bin/env python3
"""C2 (Llama-3-8B FP8_DEFAULT_CFG, 512 x 512 tokens) one-time costs: the first mtq.quantize of the
process (bench.py's order: bf16 warm-up + timed forward first) against a second one on a fresh
model in the same process, each split into phases with a device sync between them:
convert (module swap + quantizer config), weight pass + stats enable, calibration forward,
finish (amax load), validation.  Prints one JSON line."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402


def main():
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization import model_calib as MC
    from modelopt_amd.torch.quantization.config import QuantizeConfig
    from modelopt_amd.torch.quantization.conversion import replace_quant_module, set_quantizer_by_cfg
    from modelopt_amd.torch.quantization.model_quant import _validate_quantizer_attrs
    from scripts.ptq_llama import build_model

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    ids = torch.randint(0, 128256, (512, 512), device=dev, generator=g)
    batches = list(ids.split(16))

    def forward_loop(m):
        with torch.no_grad():
            for b in batches:
                m(b)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return round(time.perf_counter() - t0, 4)

    res = {}
    for run in ("first", "second"):
        model = build_model(32, dev)
        if run == "first":
            forward_loop(model)
        r = {"bf16_forward_s": timed(lambda: forward_loop(model))}
        cfg = QuantizeConfig(**mtq.FP8_DEFAULT_CFG)
        r["replace_s"] = timed(lambda: replace_quant_module(model))
        r["set_cfg_s"] = timed(lambda: set_quantizer_by_cfg(model, cfg.quant_cfg))
        r["stats_weights_s"] = timed(lambda: (MC.enable_stats_collection(model), MC.weight_only_quantize(model)))
        r["calib_forward_s"] = timed(lambda: forward_loop(model))
        r["finish_s"] = timed(lambda: MC.finish_stats_collection(model))
        r["promote_s"] = timed(lambda: MC.promote_static_block_weight_quantizers(model))
        r["validate_s"] = timed(lambda: _validate_quantizer_attrs(model))
        r["sum_s"] = round(sum(v for k, v in r.items() if k != "bf16_forward_s"), 4)
        res[run] = r
        print(run, json.dumps(r), file=sys.stderr, flush=True)
        del model
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
