#!/usr/bin/env python3
"""AWQ-lite alpha search per linear, Llama-3-8B shapes, one calibration batch (8192 tokens):
fused MFMA search (block_quant_dynamic_multi + awq_search_gemm, all 11 alphas) vs the unfused
per-alpha path (block_quant_dynamic, mul_cols, hipBLASLt F.linear, mse_accumulate).
Reports ms per linear and the search GEMM's TFLOP/s (2*M*N*K*G / kernel time) vs 2.5 PF."""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from modelopt_amd import _ext  # noqa: E402

ops = _ext.ops()
dev = torch.device("cuda")
M, G = int(sys.argv[1]) if len(sys.argv) > 1 else 8192, 11
SHAPES = {"q_proj": (4096, 4096), "k_proj": (1024, 4096), "gate_proj": (14336, 4096), "down_proj": (4096, 14336)}


def timeit(fn, iters=5):
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

    def fused():
        wq2 = ops.block_quant_dynamic_multi(w, pw, 128, 4, False, False)
        ops.awq_search_gemm(x, si, wq2, None, yref, loss)

    def gemm_only():
        ops.awq_search_gemm(x, si, wq, None, yref, loss)

    def unfused():
        for g in range(G):
            wqg = ops.block_quant_dynamic(w, pw[g], 128, 4, False, False)
            out = F.linear(ops.mul_cols(x, si[g]), wqg)
            ops.mse_accumulate(out, yref, loss, g)

    def hipblaslt_only():
        for g in range(G):
            F.linear(x, wq[g])

    flops = 2.0 * M * N * K * G
    r = {k: round(timeit(f), 3) for k, f in
         (("fused_ms", fused), ("search_gemm_ms", gemm_only), ("unfused_ms", unfused), ("hipblaslt_gemms_ms", hipblaslt_only))}
    r["search_gemm_tflops"] = round(flops / (r["search_gemm_ms"] * 1e-3) / 1e12, 1)
    r["hipblaslt_tflops"] = round(flops / (r["hipblaslt_gemms_ms"] * 1e-3) / 1e12, 1)
    r["search_gemm_frac_of_2.5PF"] = round(r["search_gemm_tflops"] / 2500, 3)
    r["speedup_vs_unfused"] = round(r["unfused_ms"] / r["fused_ms"], 3)
    res[name] = r
    print(name, r, file=sys.stderr, flush=True)
print(json.dumps({"M": M, "G": G, "shapes": res}))
