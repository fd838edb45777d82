#!/usr/bin/env python3
"""Decode-shaped QuantLinear forward: fused MFMA kernel vs the reference's unfused path.

One Llama-3-8B decoder layer's seven linears (q 4096x4096, k/v 1024x4096, o 4096x4096,
gate/up 14336x4096, down 4096x14336: 218 M weights, 436 MB bf16 -- larger than the 256 MB
Infinity Cache, so every pass streams W from HBM) at M = 1 / 4 / 16 input rows:

  fused    ops.qlinear_small_m: weight fake quant applied to the MFMA operands (one pass over W)
  grouped  the same, with q/k/v_proj as ONE ops.qlinear_small_m_group launch (what the HF
           attention wrapper runs for a decode step) and the other four linears as above
  unfused  the reference's QuantLinear forward: W_q = qdq(W) (read W, write W_q), then
           F.linear(x, W_q) on hipBLASLt (read W_q)
  bf16     F.linear(x, W) without quantization (hipBLASLt), the floor for any simulated GEMM

Reported per config and M: ms per layer (7 linears), the weight bytes / time of the fused path
as GB/s and fraction of the 8 TB/s HBM peak, and the speed-up over the unfused path.

    python scripts/bench_qlinear.py [--iters 50]
"""

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tensorrt-model-optimizer_amd"))
sys.path.insert(0, str(REPO))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = [(4096, 4096), (1024, 4096), (1024, 4096), (4096, 4096), (14336, 4096), (14336, 4096), (4096, 14336)]


GRAPH = True


def timed(fn, iters, warmup=5):
    """ms per call.  With GRAPH (default) the calls are captured once in a HIP graph and the graph
    is replayed, so host dispatch (several us per op from Python) is not in the number: the small
    k/v kernels run in less time than one eager dispatch takes."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if GRAPH:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(10):
                    fn()
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        reps = max(1, iters // 10)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / (reps * 10)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--per-linear-only", action="store_true")
    ap.add_argument("--eager", action="store_true", help="time eager launches instead of graph replays")
    ap.add_argument("--m", type=int, nargs="*", default=[1, 4, 16])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    global GRAPH
    GRAPH = not a.eager
    from modelopt_amd import _ext

    ops = _ext.ops()
    g = torch.Generator(device="cuda").manual_seed(0)
    ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16, generator=g) * 0.02 for n, k in SHAPES]
    wbytes = sum(w.numel() * 2 for w in ws)
    configs = {
        # kind, num_bits, block, amax per weight
        "int4_block128 (INT4_AWQ weights)": (0, 4, 128, [w.float().reshape(-1, 128).abs().amax(1, keepdim=True) for w in ws]),
        "fp8_per_tensor (FP8_DEFAULT weights)": (1, 8, None, [w.float().abs().amax().reshape(()) for w in ws]),
        "int8_per_channel (INT8_DEFAULT weights)": (0, 8, None, [w.float().abs().amax(1, keepdim=True) for w in ws]),
    }
    res = {"layer": "Llama-3-8B decoder layer, 7 linears, 218 M weights bf16", "weight_bytes": wbytes,
           "timing": "eager launches" if a.eager else "HIP graph replays (no host dispatch)",
           "env": {k: v for k, v in __import__("os").environ.items() if k.startswith("MTQ_AMD_QLINEAR")},
           "results": {}}
    for m in a.m:
        xs = {k: torch.randn(m, k, device="cuda", dtype=torch.bfloat16, generator=g) for k in (4096, 14336)}

        def bf16():
            for w in ws:
                F.linear(xs[w.shape[1]], w)

        t_bf16 = timed(bf16, a.iters)
        res["results"][f"M={m}"] = {"bf16_F.linear_ms": round(t_bf16, 4)}
        for name, (kind, nb, block, amaxs) in ([] if a.per_linear_only else configs.items()):
            blocks = [block or w.shape[1] for w in ws]

            def fused():
                for w, am, b in zip(ws, amaxs, blocks):
                    ops.qlinear_small_m(xs[w.shape[1]], w, None, am, b, kind, nb, False, False)

            def unfused():
                for w, am, b in zip(ws, amaxs, blocks):
                    if am.numel() == 1:
                        wq = ops.quantize_op(w, am, nb, 4 if kind else 0, False, False)
                    else:
                        wq = ops.quantize_op(w.view(-1, b), am, nb, 4 if kind else 0, False, False).view_as(w)
                    F.linear(xs[w.shape[1]], wq)

            def grouped():
                x = xs[4096]
                ops.qlinear_small_m_group([x, x, x], ws[:3], [None] * 3, amaxs[:3], blocks[:3], kind, [nb] * 3,
                                          [0] * 3, [0] * 3)
                for w, am, b in zip(ws[3:], amaxs[3:], blocks[3:]):
                    ops.qlinear_small_m(xs[w.shape[1]], w, None, am, b, kind, nb, False, False)

            def qkv_grouped():
                x = xs[4096]
                ops.qlinear_small_m_group([x, x, x], ws[:3], [None] * 3, amaxs[:3], blocks[:3], kind, [nb] * 3,
                                          [0] * 3, [0] * 3)

            def qkv_single():
                for w, am, b in zip(ws[:3], amaxs[:3], blocks[:3]):
                    ops.qlinear_small_m(xs[4096], w, None, am, b, kind, nb, False, False)

            t_f, t_u, t_g = timed(fused, a.iters), timed(unfused, a.iters), timed(grouped, a.iters)
            t_qg, t_qs = timed(qkv_grouped, a.iters), timed(qkv_single, a.iters)
            gbs = wbytes / (t_f * 1e-3) / 1e9
            gbg = wbytes / (t_g * 1e-3) / 1e9
            qkv_bytes = sum(w.numel() * 2 for w in ws[:3])
            res["results"][f"M={m}"][name] = {
                "fused_ms": round(t_f, 4), "unfused_ms": round(t_u, 4), "speedup": round(t_u / t_f, 2),
                "fused_weight_GB_s": round(gbs, 1), "fused_frac_hbm": round(gbs / 8000.0, 4),
                "grouped_qkv_layer_ms": round(t_g, 4), "grouped_weight_GB_s": round(gbg, 1),
                "grouped_frac_hbm": round(gbg / 8000.0, 4),
                "qkv_grouped_us": round(t_qg * 1e3, 2), "qkv_three_launches_us": round(t_qs * 1e3, 2),
                "qkv_grouped_GB_s": round(qkv_bytes / (t_qg * 1e-3) / 1e9, 1),
            }
        # per-linear split of the fused INT4 path (launch / latency-bound small matrices)
        for name in ("int4_block128 (INT4_AWQ weights)", "fp8_per_tensor (FP8_DEFAULT weights)"):
            kind, nb, block, amaxs = configs[name]
            per = {}
            for i, (w, am) in enumerate(zip(ws, amaxs)):
                b = block or w.shape[1]
                t = timed(lambda: ops.qlinear_small_m(xs[w.shape[1]], w, None, am, b, kind, nb, False, False), a.iters)
                per[f"{i}:{w.shape[0]}x{w.shape[1]}"] = [round(t * 1e3, 2), round(w.numel() * 2 / (t * 1e-3) / 1e9, 1)]
            res["results"][f"M={m}"][name.split()[0] + "_fused_per_linear_us_GBs"] = per
        print(json.dumps({f"M={m}": res["results"][f"M={m}"]}), flush=True)
    print(json.dumps(res))
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
