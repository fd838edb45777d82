#!/usr/bin/env python3
"""Measurement only: the 4-wave register-staged AWQ search kernel (scripts/exp/awq_w4r.hip) against
the product call (prescale + awq_search_pp_kernel) and the serial hipBLASLt path on Llama-3-8B
shapes, 8192 tokens, 11 alphas, interleaved rounds.  The variant's per-alpha losses (from its tile
partials) must match the product's within rtol 1e-4 (summation order differs)."""
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
lib = ctypes.CDLL(str(REPO / "scripts/exp/libawq_w4r.so"))
lib.awq_w4r.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                        ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
VARS = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "2"])]
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
SHAPES = {"k_proj": (1024, 4096), "q_proj": (4096, 4096), "gate_proj": (14336, 4096), "down_proj": (4096, 14336)}
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
    out_all = torch.empty(G, M, N, dtype=torch.bfloat16, device=dev)

    def var(v):
        def f():
            rc = lib.awq_w4r(v, xs.data_ptr(), wq.data_ptr(), yref.data_ptr(), part.data_ptr(), M, N, K, G, stream)
            assert rc == 0, rc
        return f

    def product():
        ops.awq_search_gemm(x, si, wq, None, yref, torch.zeros(G, device=dev))

    def serial():
        xs2 = ops.awq_prescale(x, si)
        for g in range(G):
            torch.mm(xs2[g], wq[g].t(), out=out_all[g])
        ops.awq_mse_multi(out_all, yref, torch.zeros(G, device=dev))

    l0 = torch.zeros(G, device=dev)
    ops.awq_search_gemm(x, si, wq, None, yref, l0)
    for v in VARS:
        part.fill_(float("nan"))
        var(v)()
        torch.cuda.synchronize()
        l1 = (part.view(G, tiles).double().sum(1) / (M * N)).float()
        assert torch.allclose(l0, l1, rtol=1e-4), (v, l0, l1)
    arms = {"product": product, "serial_hipblaslt": serial}
    arms.update({f"w4r_v{v}": var(v) for v in VARS})
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
        r[k] = {"ms": round(ms, 3), "tflops": round(flops / (ms * 1e-3) / 1e12, 1)}
    res[name] = r
    print(name, json.dumps(r), file=sys.stderr, flush=True)
    del out_all, wq, xs
    torch.cuda.empty_cache()
print(json.dumps(res))
