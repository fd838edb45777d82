#!/usr/bin/env python3
"""A/B of the AWQ search-kernel experiment variants (scripts/exp/awq_exp.hip: probes, raster group,
buffer-DMA) on Llama-3-8B shapes, 8192 tokens, 11 alphas, interleaved rounds in one process, beside
the product call (prescale + kernel) and the 11 hipBLASLt GEMMs.  Variant 0's loss partials are
checked equal to the product kernel's (same arithmetic, same order)."""
import ctypes
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from modelopt_amd import _ext  # noqa: E402

ops = _ext.ops()
lib = ctypes.CDLL(str(REPO / "scripts/exp/libawq_exp.so"))
lib.awq_exp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                        ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
w4 = ctypes.CDLL(str(REPO / "scripts/exp/libawq_w4asm.so"))
w4.awq_w4asm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
VARS = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "31,34,35,50,53".split(","))]
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
SHAPES = {"k_proj": (1024, 4096), "q_proj": (4096, 4096), "gate_proj": (14336, 4096), "down_proj": (4096, 14336)}
if len(sys.argv) > 3:  # e.g. "q_proj=4096x4096,q_k2=4096x8192"
    SHAPES = {kv.split("=")[0]: tuple(int(v) for v in kv.split("=")[1].split("x")) for kv in sys.argv[3].split(",")}
M, G = 8192, 11
dev = torch.device("cuda")
stream = torch.cuda.current_stream().cuda_stream
res = {}
for name, (N, K) in SHAPES.items():
    gen = torch.Generator(device=dev).manual_seed(N + K)
    x = torch.randn(M, K, device=dev, generator=gen).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
    s = torch.rand(G, K, device=dev, generator=gen) * 3 + 0.25
    pw, si = s.to(torch.bfloat16), (1 / s).to(torch.bfloat16)
    yref = F.linear(x, w)
    wq = ops.block_quant_dynamic_multi(w, pw, 128, 4, False, False)
    xs = ops.awq_prescale(x, si)
    tiles = (M // 256) * (N // 256)
    part = torch.zeros(G * tiles, device=dev)
    loss = torch.zeros(G, device=dev)

    def var(v):
        def f():
            if 70 <= v < 80:  # scripts/exp/awq_w4asm.hip, variant v - 70
                rc = w4.awq_w4asm(v - 70, xs.data_ptr(), wq.data_ptr(), yref.data_ptr(), part.data_ptr(), M, N, K, G, stream)
            else:
                rc = lib.awq_exp(v, xs.data_ptr(), wq.data_ptr(), yref.data_ptr(), part.data_ptr(), M, N, K, G, stream)
            assert rc == 0, rc
        return f

    def product():
        ops.awq_search_gemm(x, si, wq, None, yref, loss)

    def product_pp():
        ops.awq_search_gemm(x, si, wq, None, yref, loss, 1)

    def prescale():
        ops.awq_prescale(x, si)

    def gemms():
        for g in range(G):
            F.linear(xs[g], wq[g])

    # correctness of the copy: variant 0's per-alpha loss equals the product's
    l0 = torch.zeros(G, device=dev)
    ops.awq_search_gemm(x, si, wq, None, yref, l0)
    for v in [0] + [v for v in VARS if v in (10, 20, 21, 22, 30, 31, 34, 50) or 70 <= v < 73]:
        part.fill_(float("nan"))
        var(v)()
        torch.cuda.synchronize()
        l1 = (part.view(G, tiles).double().sum(1) / (M * N)).float()
        if not torch.allclose(l0, l1, rtol=1e-5):
            print(f"{name}: variant {v} loss MISMATCH {l0.tolist()[:3]} vs {l1.tolist()[:3]}", file=sys.stderr, flush=True)
            assert v != 0
    arms = {"product": product, "product_pp": product_pp, "prescale": prescale, "hipblaslt_gemms": gemms}
    arms.update({f"v{v}": var(v) for v in VARS})
    t = {k: [] for k in arms}
    for _ in range(ROUNDS):
        for k, f in arms.items():
            f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f()
            e1.record()
            torch.cuda.synchronize()
            t[k].append(e0.elapsed_time(e1) / 3)
    flops = 2.0 * M * N * K * G
    r = {}
    for k, v in t.items():
        ms = statistics.median(v)
        r[k] = {"ms": round(ms, 3), "min_ms": round(min(v), 3), "tflops": round(flops / (ms * 1e-3) / 1e12, 1)}
    res[name] = r
    print(name, json.dumps(r), file=sys.stderr, flush=True)
print(json.dumps(res))
