#!/usr/bin/env python3
"""AWQ-lite alpha search per linear, Llama-3-8B shapes, one calibration batch (8192 tokens, 11
alphas), all in one process with interleaved rounds (cdna_hip_programming.md §5.4 rule 24):

* ``fused``   -- mtq_awq_search_gemm: the pre-scale pass + the MFMA search kernel with the loss in
                 its epilogue (the r06 one-wave-per-SIMD kernel where K >= 128)
* ``fused_pp`` -- the same with the r03 ping-pong kernel (kernel=1)
* ``batched`` -- the wide-linear path: awq_prescale + 11 hipBLASLt torch.mm into [G, M, N] +
                 awq_mse_multi
* ``per_alpha`` -- the r01 path: per alpha mul_cols + hipBLASLt F.linear + mse_accumulate
* ``hipblaslt_gemms`` -- the 11 bf16 GEMMs alone
Reports ms (median over rounds) and TFLOP/s = 2*M*N*K*G / time vs the 2.5 PF dense bf16 peak.
Usage: bench_awq_gemm.py [M] [rounds]"""
import json
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
    loss = torch.zeros(G, device=dev)
    wq = ops.block_quant_dynamic_multi(w, pw, 128, 4, False, False)

    def search():
        ops.awq_search_gemm(x, si, wq, None, yref, loss)

    def search_pp():
        ops.awq_search_gemm(x, si, wq, None, yref, loss, 1)

    def batched():
        xs = ops.awq_prescale(x, si)
        out = torch.empty((G, M, N), dtype=x.dtype, device=dev)
        for g in range(G):
            torch.mm(xs[g], wq[g].t(), out=out[g])
        ops.awq_mse_multi(out, yref, loss)

    def per_alpha():
        for g in range(G):
            out = F.linear(ops.mul_cols(x, si[g]), wq[g])
            ops.mse_accumulate(out, yref, loss, g)

    def hipblaslt_gemms():
        for g in range(G):
            F.linear(x, wq[g])

    arms = {"fused": search, "fused_pp": search_pp, "batched": batched, "per_alpha": per_alpha, "hipblaslt_gemms": hipblaslt_gemms}
    t = {k: [] for k in arms}
    names = list(arms)
    for r_ in range(ROUNDS):  # rotated order per round: a fixed order biases an arm by ~4 %
        for k in names[r_ % len(names):] + names[:r_ % len(names)]:
            t[k].append(timeit(arms[k]))
    flops = 2.0 * M * N * K * G
    r = {}
    for k, v in t.items():
        ms = statistics.median(v)
        r[k] = {"ms": round(ms, 3), "min_ms": round(min(v), 3), "tflops": round(flops / (ms * 1e-3) / 1e12, 1)}
        r[k]["frac_of_2.5PF"] = round(r[k]["tflops"] / 2500, 3)
    r["fused_speedup_vs_batched"] = round(r["batched"]["ms"] / r["fused"]["ms"], 3)
    r["fused_speedup_vs_per_alpha"] = round(r["per_alpha"]["ms"] / r["fused"]["ms"], 3)
    res[name] = r
    print(name, json.dumps(r), file=sys.stderr, flush=True)
print(json.dumps({"M": M, "G": G, "rounds": ROUNDS, "shapes": res}))
