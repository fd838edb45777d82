#!/usr/bin/env python3
"""End-to-end PTQ wall-clock: mtq.quantize(Llama-3-8B | Mixtral-8x7B, FP8_DEFAULT_CFG, 512 x 512 tokens).

SURVEY.md §8d (E2E): LlamaForCausalLM built from the Llama-3-8B config (random bf16 weights, no
checkpoint -- there is no network), 512 samples x 512 token ids uniform in [0, 128256) (seed 1234),
batch 16, timer = mtq.quantize entry -> return with the model already on the device.  With
torch.distributed initialised each rank calibrates samples/world (DP) and the amax exchange is the
one packed all_reduce(MAX).  Also times the same forward passes without quantizers, so the
quantizer overhead on top of the bf16 GEMMs is visible.

C5 (``--model mixtral-8x7b``): Mixtral-8x7B dims (transformers-5 fused experts, 8 experts top-2,
46.7 G params = 93 GB bf16, resident on one GPU), same calibration set (vocab 32000).

    python benchmarks/ptq_llama.py [--model llama3-8b] [--layers 32] [--samples 512] [--seq 512] [--batch 16]
"""

from __future__ import annotations

import argparse
import gc
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
for p in (str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

LLAMA3_8B = dict(
    hidden_size=4096,
    intermediate_size=14336,
    num_hidden_layers=32,
    num_attention_heads=32,
    num_key_value_heads=8,
    vocab_size=128256,
    max_position_embeddings=8192,
    rope_theta=500000.0,
    rms_norm_eps=1e-5,
)

MIXTRAL_8X7B = dict(
    hidden_size=4096,
    intermediate_size=14336,
    num_hidden_layers=32,
    num_attention_heads=32,
    num_key_value_heads=8,
    vocab_size=32000,
    max_position_embeddings=32768,
    rope_theta=1e6,
    rms_norm_eps=1e-5,
    num_local_experts=8,
    num_experts_per_tok=2,
)
MODELS = {"llama3-8b": ("Llama-3-8B", LLAMA3_8B), "mixtral-8x7b": ("Mixtral-8x7B", MIXTRAL_8X7B)}


def build_model(layers: int, device, model="llama3-8b"):
    from transformers import LlamaConfig, LlamaForCausalLM, MixtralConfig, MixtralForCausalLM

    dims = MODELS[model][1]
    cfg_cls, model_cls = (MixtralConfig, MixtralForCausalLM) if model.startswith("mixtral") else (LlamaConfig, LlamaForCausalLM)
    cfg = cfg_cls(**{**dims, "num_hidden_layers": layers})
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(1234)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device(device):
            model = model_cls(cfg)
    finally:
        torch.set_default_dtype(prev)
    return model.eval()


def run(samples=512, seq=512, batch=16, layers=32, config="FP8_DEFAULT_CFG", rank=0, world=1, baseline=True,
        model_name="llama3-8b", algorithm=None, kv=None):
    import modelopt_amd.torch.quantization as mtq

    dev = torch.device("cuda", torch.cuda.current_device())
    model = build_model(layers, dev, model_name)
    if model_name.startswith("mixtral"):
        # the bf16 baseline runs the same eager expert loop the quantized experts intercept
        model.config._experts_implementation = "eager"
    label, dims = MODELS[model_name]
    g = torch.Generator(device=dev).manual_seed(1234)
    ids = torch.randint(0, dims["vocab_size"], (samples, seq), device=dev, generator=g)
    per = samples // world
    mine = ids[rank * per : (rank + 1) * per]
    batches = list(mine.split(batch))

    passes = []  # (start, end) of every forward_loop call

    def forward_loop(m):
        t = time.perf_counter()
        with torch.no_grad():
            for b in batches:
                m(b)
        torch.cuda.synchronize()
        passes.append((t, time.perf_counter()))

    gc_events = []

    def _gc_cb(phase, info):  # cyclic-GC collections inside the timed regions (host time)
        if phase == "start":
            gc_events.append([info["generation"], time.perf_counter(), None])
        elif gc_events and gc_events[-1][2] is None:
            gc_events[-1][2] = time.perf_counter()

    def gc_summary(t0, t1):
        ev = [e for e in gc_events if e[2] is not None and t0 <= e[1] <= t1]
        return {f"gen{g}": {"n": sum(1 for e in ev if e[0] == g),
                            "s": round(sum(e[2] - e[1] for e in ev if e[0] == g), 4)} for g in (0, 1, 2)}

    res = {"model": f"{label} dims, {layers} layers, bf16 random init", "samples": samples,
           "seq": seq, "batch": batch, "world": world, "config": config}
    # Both timed regions start from a collected Python heap: building a 16-140 GB HF model leaves a
    # generation-2 collection due (0.16 s on a 436 k-object heap, profiles/r04/ptq/c2_gc_r04zc.json)
    # that otherwise fires inside whichever timed region allocates next -- the model build's debt,
    # not quantization work.
    if baseline:
        forward_loop(model)  # warm-up (kernels, allocator)
        gc.collect()
        torch.cuda.synchronize()
        gc.callbacks.append(_gc_cb)
        t0 = time.perf_counter()
        forward_loop(model)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        gc.callbacks.remove(_gc_cb)
        res["bf16_forward_s"] = round(t1 - t0, 3)
        res["bf16_gc"] = gc_summary(t0, t1)
    gc.collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cfg = getattr(mtq, config)
    if algorithm is not None or kv is not None:
        import copy

        cfg = copy.deepcopy(cfg)
    if algorithm is not None:
        cfg["algorithm"] = algorithm
        res["algorithm"] = algorithm
    if kv is not None:  # e.g. FP8_KV_CFG: K/V cache fake quant inside every attention
        cfg["quant_cfg"] = cfg["quant_cfg"] + getattr(mtq, kv)["quant_cfg"]
        res["kv"] = kv
    gc.callbacks.append(_gc_cb)
    passes.clear()
    mtq.quantize(model, cfg, forward_loop)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    gc.callbacks.remove(_gc_cb)
    res["ptq_wall_clock_s"] = round(t1 - t0, 3)
    if len(passes) == 1:  # one calibration pass (max): where the time outside the forward goes
        (p0, p1), = passes
        res["ptq_phases_s"] = {"before_first_batch": round(p0 - t0, 4), "calibration_forward": round(p1 - p0, 4),
                               "after_last_batch": round(t1 - p1, 4)}
    res["ptq_gc"] = gc_summary(t0, t1)
    n_q = sum(1 for _, m in model.named_modules() if isinstance(m, mtq.TensorQuantizer) and m.is_enabled)
    res["enabled_quantizers"] = n_q
    if baseline:
        res["quantizer_overhead_s"] = round(res["ptq_wall_clock_s"] - res["bf16_forward_s"], 3)
    tok = samples * seq
    res["calib_tokens_per_s"] = round(tok / res["ptq_wall_clock_s"], 1)
    # sanity: quantized forward is finite
    with torch.no_grad():
        out = model(batches[0][:1, :64]).logits
    res["finite_logits"] = bool(torch.isfinite(out).all())
    del model
    torch.cuda.empty_cache()
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b", choices=sorted(MODELS))
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--samples", type=int, default=512)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--config", default="FP8_DEFAULT_CFG")
    ap.add_argument("--no-baseline", action="store_true")
    ap.add_argument("--kv", default=None, help="KV preset appended to the config, e.g. FP8_KV_CFG")
    ap.add_argument("--algorithm", default=None, help='JSON override, e.g. \'{"method": "awq_full"}\'')
    a = ap.parse_args()
    algo = json.loads(a.algorithm) if a.algorithm else None
    print(json.dumps(run(a.samples, a.seq, a.batch, a.layers, a.config, baseline=not a.no_baseline,
                         model_name=a.model, algorithm=algo, kv=a.kv)), flush=True)
