#!/usr/bin/env python3
"""Measurement only: the wide-linear AWQ search path (model_calib._awq_search_fast, N > 2048) with
its HBM-bound passes overlapped with the hipBLASLt GEMMs on a second stream, against the current
serial form and the fused MFMA kernel.  Llama-3-8B shapes, 8192 tokens, 11 alphas, interleaved rounds.

arms:
  serial   prescale(all alphas) -> 11 x torch.mm into [G, M, N] -> awq_mse_multi(all)   (product today)
  ovl_mse  prescale(all) -> mm g on the main stream, mse of alpha g on a side stream (2 output slots)
  ovl_all  prescale of alpha g+1 and the loss pass of alpha g-1 on a side stream beside mm g
           (two slots each; the form r04e measured, profiles/r04/awq/overlap_ab_r04e.json)
  fused    ops.awq_search_gemm (prescale + MFMA kernel with the loss in the epilogue)
The per-alpha losses of every overlapped arm must equal the serial arm's bit for bit (same kernels,
same per-alpha reduction order)."""
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from modelopt_amd import _ext  # noqa: E402

ops = _ext.ops()
ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
SHAPES = {"k_proj": (1024, 4096), "q_proj": (4096, 4096), "gate_proj": (14336, 4096), "down_proj": (4096, 14336)}
M, G = 8192, 11
dev = torch.device("cuda")
side = torch.cuda.Stream()
res = {}
for name, (N, K) in SHAPES.items():
    gen = torch.Generator(device=dev).manual_seed(N + K)
    x = torch.randn(M, K, device=dev, generator=gen).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
    s = torch.rand(G, K, device=dev, generator=gen) * 3 + 0.25
    pw, si = s.to(torch.bfloat16), (1 / s).to(torch.bfloat16)
    yref = torch.nn.functional.linear(x, w)
    wq = ops.block_quant_dynamic_multi(w, pw, 128, 4, False, False)
    out_all = torch.empty(G, M, N, dtype=torch.bfloat16, device=dev)
    slots = torch.empty(2, M, N, dtype=torch.bfloat16, device=dev)

    def serial(loss):
        xs = ops.awq_prescale(x, si)
        for g in range(G):
            torch.mm(xs[g], wq[g].t(), out=out_all[g])
        ops.awq_mse_multi(out_all, yref, loss)

    def ovl_mse(loss):
        main = torch.cuda.current_stream()
        xs = ops.awq_prescale(x, si)
        done = [torch.cuda.Event(), torch.cuda.Event()]  # slot free again (mse of it finished)
        for g in range(G):
            sl = g & 1
            if g >= 2:
                main.wait_event(done[sl])
            torch.mm(xs[g], wq[g].t(), out=slots[sl])
            ev = torch.cuda.Event()
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                ops.awq_mse_multi(slots[sl][None], yref, loss[g:g + 1])
                done[sl].record(side)
        main.wait_stream(side)

    xs_slots = torch.empty(2, 1, M, K, dtype=torch.bfloat16, device=dev)

    def ovl_all(loss):
        main = torch.cuda.current_stream()
        ev_xs = [torch.cuda.Event(), torch.cuda.Event()]
        ev_mm = [torch.cuda.Event(), torch.cuda.Event()]
        ev_mse = [torch.cuda.Event(), torch.cuda.Event()]
        side.wait_stream(main)
        with torch.cuda.stream(side):
            xs_slots[0].copy_(ops.awq_prescale(x, si[0:1]))
            ev_xs[0].record(side)
        for g in range(G):
            sl = g & 1
            if g + 1 < G:
                with torch.cuda.stream(side):
                    if g >= 1:
                        side.wait_event(ev_mm[1 - sl])
                    xs_slots[1 - sl].copy_(ops.awq_prescale(x, si[g + 1:g + 2]))
                    ev_xs[1 - sl].record(side)
            main.wait_event(ev_xs[sl])
            if g >= 2:
                main.wait_event(ev_mse[sl])
            torch.mm(xs_slots[sl, 0], wq[g].t(), out=slots[sl])
            ev_mm[sl].record(main)
            with torch.cuda.stream(side):
                side.wait_event(ev_mm[sl])
                ops.awq_mse_multi(slots[sl:sl + 1], yref, loss[g:g + 1])
                ev_mse[sl].record(side)
        main.wait_stream(side)

    def fused(loss):
        ops.awq_search_gemm(x, si, wq, None, yref, loss)

    arms = {"serial": serial, "ovl_mse": ovl_mse, "ovl_all": ovl_all, "fused": fused}
    ref_loss = torch.zeros(G, device=dev)
    serial(ref_loss)
    torch.cuda.synchronize()
    for k in ("ovl_mse", "ovl_all"):
        lo = torch.zeros(G, device=dev)
        arms[k](lo)
        torch.cuda.synchronize()
        assert torch.equal(lo, ref_loss), (k, lo, ref_loss)
    t = {k: [] for k in arms}
    loss = torch.zeros(G, device=dev)
    for _ in range(ROUNDS):
        for k, f in arms.items():
            f(loss)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f(loss)
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
    del out_all, slots, xs_slots, wq
    torch.cuda.empty_cache()
print(json.dumps(res))
