#!/usr/bin/env python3
"""AWQ-lite alpha search per linear, Llama-3-8B shapes, one calibration batch (8192 tokens, 11
alphas), all in one process with interleaved rounds (cdna_hip_programming.md §5.4 rule 24):

* ``pp5``     -- mtq_awq_search_gemm mode 2, default schedule 5 (r03 ping-pong kernel + pre-scale
                 pass; B0 fragments held in registers, every half-tile issued 4-5 phases ahead)
* ``pp4``     -- schedule 4 (the first r03 schedule, fragments re-read per phase); ``pp4_branch``
                 the same with the last tile's loads skipped behind a branch (MTQ_AMD_AWQ_PP_CLAMP=0)
* ``w4``      -- schedule 6: four waves, one per SIMD, 128 x 128 per wave, one barrier per K tile
* ``*_noload_probe`` -- pp5 / pp4 without global loads in the K loop (skeleton timing; wrong losses)
* ``r02``     -- mode 1 (r02 kernel, x scaled while register-staged)
* ``batched`` -- the r02 wide-linear path: awq_prescale + 11 hipBLASLt torch.mm into [G, M, N] +
                 awq_mse_multi
* ``per_alpha`` -- the r01 path: per alpha mul_cols + hipBLASLt F.linear + mse_accumulate
* ``hipblaslt_gemms`` -- the 11 bf16 GEMMs alone
Reports ms (median over rounds) and TFLOP/s = 2*M*N*K*G / time vs the 2.5 PF dense bf16 peak.
Usage: bench_awq_gemm.py [M] [rounds]"""
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


def with_mode(mode, fn, phases=5, probe=0, clamp=1):
    def run():
        os.environ["MTQ_AMD_AWQ_PP_CLAMP"] = str(clamp)
        os.environ["MTQ_AMD_AWQ_GEMM_MODE"] = str(mode)
        os.environ["MTQ_AMD_AWQ_PP_PHASES"] = str(phases)
        os.environ["MTQ_AMD_AWQ_GEMM_PROBE"] = str(probe)
        fn()
    return run


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

    arms = {"pp5": with_mode(2, search), "pp4": with_mode(2, search, 4),
            "pp4_branch": with_mode(2, search, 4, clamp=0), "w4": with_mode(2, search, 6),
            "pp5_noload_probe": with_mode(2, search, 5, 1), "pp4_noload_probe": with_mode(2, search, 4, 1),
            "r02": with_mode(1, search), "batched": batched,
            "per_alpha": per_alpha, "hipblaslt_gemms": hipblaslt_gemms}
    t = {k: [] for k in arms}
    for _ in range(ROUNDS):
        for k, f in arms.items():
            t[k].append(timeit(f))
    flops = 2.0 * M * N * K * G
    r = {}
    for k, v in t.items():
        ms = statistics.median(v)
        r[k] = {"ms": round(ms, 3), "min_ms": round(min(v), 3), "tflops": round(flops / (ms * 1e-3) / 1e12, 1)}
        r[k]["frac_of_2.5PF"] = round(r[k]["tflops"] / 2500, 3)
    r["pp5_speedup_vs_batched"] = round(r["batched"]["ms"] / r["pp5"]["ms"], 3)
    r["pp5_speedup_vs_per_alpha"] = round(r["per_alpha"]["ms"] / r["pp5"]["ms"], 3)
    r["pp5_speedup_vs_r02"] = round(r["r02"]["ms"] / r["pp5"]["ms"], 3)
    r["w4_speedup_vs_pp5"] = round(r["pp5"]["ms"] / r["w4"]["ms"], 3)
    res[name] = r
    print(name, json.dumps(r), file=sys.stderr, flush=True)
os.environ.pop("MTQ_AMD_AWQ_GEMM_MODE", None)
os.environ.pop("MTQ_AMD_AWQ_PP_PHASES", None)
os.environ.pop("MTQ_AMD_AWQ_GEMM_PROBE", None)
os.environ.pop("MTQ_AMD_AWQ_PP_CLAMP", None)
print(json.dumps({"M": M, "G": G, "rounds": ROUNDS, "shapes": res}))
