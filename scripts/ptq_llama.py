#!/usr/bin/env python3
"""End-to-end PTQ wall-clock: mtq.quantize(Llama-3-8B, FP8_DEFAULT_CFG, 512 x 512 synthetic tokens).

SURVEY.md §8d (E2E): LlamaForCausalLM built from the Llama-3-8B config (random bf16 weights, no
checkpoint -- there is no network), 512 samples x 512 token ids uniform in [0, 128256) (seed 1234),
batch 16, timer = mtq.quantize entry -> return with the model already on the device.  With
torch.distributed initialised each rank calibrates samples/world (DP) and the amax exchange is the
one packed all_reduce(MAX).  Also times the same forward passes without quantizers, so the
quantizer overhead on top of the bf16 GEMMs is visible.

    python scripts/ptq_llama.py [--layers 32] [--samples 512] [--seq 512] [--batch 16]
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


def build_model(layers: int, device):
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(**{**LLAMA3_8B, "num_hidden_layers": layers})
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(1234)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device(device):
            model = LlamaForCausalLM(cfg)
    finally:
        torch.set_default_dtype(prev)
    return model.eval()


def run(samples=512, seq=512, batch=16, layers=32, config="FP8_DEFAULT_CFG", rank=0, world=1, baseline=True):
    import modelopt_amd.torch.quantization as mtq

    dev = torch.device("cuda", torch.cuda.current_device())
    model = build_model(layers, dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    ids = torch.randint(0, LLAMA3_8B["vocab_size"], (samples, seq), device=dev, generator=g)
    per = samples // world
    mine = ids[rank * per : (rank + 1) * per]
    batches = list(mine.split(batch))

    def forward_loop(m):
        with torch.no_grad():
            for b in batches:
                m(b)

    res = {"model": f"Llama-3-8B dims, {layers} layers, bf16 random init", "samples": samples,
           "seq": seq, "batch": batch, "world": world, "config": config}
    if baseline:
        forward_loop(model)  # warm-up (kernels, allocator)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        forward_loop(model)
        torch.cuda.synchronize()
        res["bf16_forward_s"] = round(time.perf_counter() - t0, 3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mtq.quantize(model, getattr(mtq, config), forward_loop)
    torch.cuda.synchronize()
    res["ptq_wall_clock_s"] = round(time.perf_counter() - t0, 3)
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
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--samples", type=int, default=512)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--config", default="FP8_DEFAULT_CFG")
    ap.add_argument("--no-baseline", action="store_true")
    a = ap.parse_args()
    print(json.dumps(run(a.samples, a.seq, a.batch, a.layers, a.config, baseline=not a.no_baseline)), flush=True)
