#!/usr/bin/env python3
"""Host profile of the one-time phases of mtq.quantize around the calibration forward: before the
first batch (conversion, weight amax pass) and after the last (amax load, checks, promotion).  Their
cost scales with the number of quantizers, not with the tensor sizes, so a narrow model with the
real layer / expert counts reproduces it: Mixtral-8x7B's 32 layers x 8 experts (1094 quantizers) or
Llama-3-8B's 32 layers at hidden 256.  Prints the wall time of each phase and the cProfile top of
each.   python scripts/prof_ptq_phases.py [mixtral|llama] [hidden]"""
import cProfile
import io
import json
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

import modelopt_amd.torch.quantization as mtq  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "mixtral"
hidden = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def build():
    from transformers import LlamaConfig, LlamaForCausalLM, MixtralConfig, MixtralForCausalLM

    common = dict(hidden_size=hidden, intermediate_size=2 * hidden, num_hidden_layers=32, num_attention_heads=8,
                  num_key_value_heads=2, vocab_size=512)
    if kind == "mixtral":
        cfg = MixtralConfig(**common, num_local_experts=8, num_experts_per_tok=2)
    else:
        cfg = LlamaConfig(**common)
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(0)
    m = (MixtralForCausalLM if kind == "mixtral" else LlamaForCausalLM)(cfg).eval().to(torch.bfloat16).to(dev)
    if kind == "mixtral":
        m.config._experts_implementation = "eager"
    return m


ids = [torch.randint(0, 512, (4, 64), device=dev) for _ in range(2)]


def top(pr, n=25):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(n)
    return s.getvalue()


res = {}
for rnd in range(3):  # rounds 1-2: steady state (first-use costs paid); round 2 under cProfile
    model = build()
    with torch.no_grad():
        model(ids[0])
    if dev.type == "cuda":
        torch.cuda.synchronize()
    pre, post = cProfile.Profile(), cProfile.Profile()
    marks = {}

    prof = rnd == 2

    def loop(m):
        pre.disable()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        marks["loop0"] = time.perf_counter()
        with torch.no_grad():
            for b in ids:
                m(b)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        marks["loop1"] = time.perf_counter()
        if prof:
            post.enable()

    t0 = time.perf_counter()
    if prof:
        pre.enable()
    mtq.quantize(model, mtq.FP8_DEFAULT_CFG, loop)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    post.disable()
    res[f"round{rnd}"] = {"before_first_batch_s": round(marks["loop0"] - t0, 4),
                          "after_last_batch_s": round(t1 - marks["loop1"], 4)}
    if prof:
        print("=== before first batch (profiled)\n" + top(pre), file=sys.stderr)
        print("=== after last batch (profiled)\n" + top(post), file=sys.stderr)
    del model
print(json.dumps({"model": kind, "hidden": hidden, **res}))
