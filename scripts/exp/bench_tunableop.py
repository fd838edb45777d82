#!/usr/bin/env python3
"""Measurement only: the AWQ search's per-alpha GEMMs (torch.mm of xs[g] [M, K] by wq[g]^T into a
[G, M, N] slice, model_calib wide path) under PyTorch's default hipBLASLt heuristic against the
solution TunableOp picks for the same shape, on Llama-3-8B shapes, 8192 tokens, 11 alphas."""
import json
import os
import statistics
import sys
import time

import torch

M, G = 8192, 11
SHAPES = {"k_proj": (1024, 4096), "q_proj": (4096, 4096), "gate_proj": (14336, 4096), "down_proj": (4096, 14336)}
ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda")
os.makedirs("gpurun_out", exist_ok=True)


def timed(f, reps=3):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


tun = torch.cuda.tunable
res = {}
for name, (N, K) in SHAPES.items():
    gen = torch.Generator(device=dev).manual_seed(N + K)
    xs = torch.randn(G, M, K, device=dev, generator=gen).to(torch.bfloat16)
    wq = (torch.randn(G, N, K, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
    out = torch.empty(G, M, N, dtype=torch.bfloat16, device=dev)

    def run():
        for g in range(G):
            torch.mm(xs[g], wq[g].t(), out=out[g])

    tun.enable(False)
    ref = None
    run()
    torch.cuda.synchronize()
    ref = out.clone()
    tun.enable(True)
    tun.tuning_enable(True)
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    tune_s = time.perf_counter() - t0
    tun.tuning_enable(False)
    diff = (out.float() - ref.float()).abs().max().item()
    t = {"default": [], "tuned": []}
    for _ in range(ROUNDS):
        tun.enable(False)
        t["default"].append(timed(run))
        tun.enable(True)
        t["tuned"].append(timed(run))
    flops = 2.0 * M * N * K * G
    r = {k: {"ms": round(statistics.median(v), 3), "tflops": round(flops / (statistics.median(v) * 1e-3) / 1e12, 1)}
         for k, v in t.items()}
    r["tune_s"] = round(tune_s, 1)
    r["max_abs_diff_vs_default"] = diff
    res[name] = r
    print(name, json.dumps(r), file=sys.stderr, flush=True)
    del xs, wq, out, ref
    torch.cuda.empty_cache()
print(json.dumps(res))
