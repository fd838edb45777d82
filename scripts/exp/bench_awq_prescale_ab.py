#!/usr/bin/env python3
"""A/B of the fused AWQ search with the x * (1/s) pre-scale pass (xs [G, M, K] written, then read
by the search kernel) against the in-kernel scaling of the X fragments (r05), interleaved in one
process, Llama-3-8B shapes, 11 alphas; the batched hipBLASLt path beside them.  The two fused forms
must give bit-identical losses.   python scripts/bench_awq_prescale_ab.py [M] [rounds]"""
import json
import os
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from modelopt_amd import _ext  # noqa: E402

ops = _ext.ops()
dev = torch.device("cuda")
M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
G = 11
SHAPES = {"k_proj": (1024, 4096), "q_proj": (4096, 4096), "gate_proj": (14336, 4096), "down_proj": (4096, 14336)}


def timeit(fn, iters=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


res = {}
for name, (N, K) in SHAPES.items():
    gen = torch.Generator(device=dev).manual_seed(N + K)
    x = torch.randn(M, K, device=dev, generator=gen).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
    s = torch.rand(G, K, device=dev, generator=gen) * 3 + 0.25
    pw, si = s.to(torch.bfloat16), (1 / s).to(torch.bfloat16)
    yref = F.linear(x, w)
    wq = ops.block_quant_dynamic_multi(w, pw, 128, 4, False, False)
    losses = {}

    def fused(flag):
        def f():
            os.environ["MTQ_AMD_AWQ_PRESCALE_EXP"] = flag
            loss = torch.zeros(G, device=dev)
            ops.awq_search_gemm(x, si, wq, None, yref, loss)
            losses[flag] = loss
        return f

    def batched():
        xs = ops.awq_prescale(x, si)
        out = torch.empty(G, M, N, device=dev, dtype=torch.bfloat16)
        for g in range(G):
            torch.mm(xs[g], wq[g].t(), out=out[g])
        loss = torch.zeros(G, device=dev)
        ops.awq_mse_multi(out, yref, loss)

    t = {"prescale": [], "inkernel": [], "batched": []}
    for _ in range(ROUNDS):
        t["prescale"].append(timeit(fused("1")))
        t["inkernel"].append(timeit(fused("0")))
        t["batched"].append(timeit(batched))
    med = {k: round(statistics.median(v), 4) for k, v in t.items()}
    flops = 2 * M * N * K * G
    res[name] = {"ms": med, "pflops": {k: round(flops / (v * 1e-3) / 1e15, 3) for k, v in med.items()},
                 "losses_equal": bool(torch.equal(losses["1"], losses["0"]))}
    print(name, json.dumps(res[name]), flush=True)
    del x, w, wq, yref
    torch.cuda.empty_cache()
os.environ.pop("MTQ_AMD_AWQ_PRESCALE_EXP", None)
print(json.dumps(res))
