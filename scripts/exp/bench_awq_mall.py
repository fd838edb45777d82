#!/usr/bin/env python3
"""Measurement only: orderings of the wide-linear AWQ search (model_calib._awq_search_fast, N > 2048)
on Llama-3-8B shapes, 8192 tokens, 11 alphas, interleaved rounds; all arms give the same losses bit
for bit (same kernels, same operands).
  serial:    x * (1/s) for all alphas [G, M, K] -> G GEMMs into [G, M, N] -> one loss pass (product)
  interleave: per alpha, x * (1/s_g) into one reused [M, K] buffer (stays in the 256 MB Infinity
             Cache for the GEMM that reads it) -> GEMM g into [G, M, N] -> one loss pass
  per_alpha: per alpha, x * (1/s_g) -> GEMM into one reused [M, N] -> loss of alpha g"""
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
res = {}
for name, (N, K) in SHAPES.items():
    gen = torch.Generator(device=dev).manual_seed(N + K)
    x = torch.randn(M, K, device=dev, generator=gen).to(torch.bfloat16)
    wq = (torch.randn(G, N, K, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
    s = torch.rand(G, K, device=dev, generator=gen) * 3 + 0.25
    si = (1 / s).to(torch.bfloat16)
    yref = torch.nn.functional.linear(x, wq[0])
    out_all = torch.empty(G, M, N, dtype=torch.bfloat16, device=dev)
    out1 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    losses = {}

    def serial(loss):
        xs = ops.awq_prescale(x, si)
        for g in range(G):
            torch.mm(xs[g], wq[g].t(), out=out_all[g])
        del xs
        ops.awq_mse_multi(out_all, yref, loss)

    def interleave(loss):
        for g in range(G):
            xg = ops.awq_prescale(x, si[g : g + 1])
            torch.mm(xg[0], wq[g].t(), out=out_all[g])
        ops.awq_mse_multi(out_all, yref, loss)

    def per_alpha(loss):
        for g in range(G):
            xg = ops.awq_prescale(x, si[g : g + 1])
            torch.mm(xg[0], wq[g].t(), out=out1)
            ops.mse_accumulate(out1, yref, loss, g)

    arms = {"serial": serial, "interleave": interleave, "per_alpha": per_alpha}
    for k, f in arms.items():
        loss = torch.zeros(G, device=dev)
        f(loss)
        torch.cuda.synchronize()
        losses[k] = loss
    for k in arms:
        assert torch.allclose(losses[k], losses["serial"], rtol=1e-5, atol=0), (k, losses[k], losses["serial"])
    t = {k: [] for k in arms}
    for _ in range(ROUNDS):
        for k, f in arms.items():
            loss = torch.zeros(G, device=dev)
            f(loss)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f(loss)
            e1.record()
            torch.cuda.synchronize()
            t[k].append(e0.elapsed_time(e1) / 3)
    res[name] = {k: round(statistics.median(v), 3) for k, v in t.items()}
    res[name]["loss_equal"] = {k: bool(torch.equal(losses[k], losses["serial"])) for k in arms}
    print(name, json.dumps(res[name]), file=sys.stderr, flush=True)
    del out_all, out1, wq
    torch.cuda.empty_cache()
print(json.dumps(res))
