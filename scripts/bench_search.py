#!/usr/bin/env python3
"""Throughput of the calibration-search kernels (csrc/mtq_search.hip) on Llama-3-8B-sized weights.

These kernels are VALU-bound (every weight element is quantised once per candidate), so beside
the HIP-event time each line reports the work rate in the kernel's own unit and, when a
``--pmc`` pass of rocprofv3 has been collected (``SQ_INSTS_VALU``), the VALU issue rate against
the MI355X peak (256 CUs x 4 SIMDs x 64 lanes / 2 cycles x 2.4 GHz = 78.6 T lane-instructions/s).

    python scripts/bench_search.py [--out profiles/r01/search.json] [--cpu]

Shapes: gate_proj [14336, 4096] bf16 (NVFP4 FP8-scale sweep, 126 candidates; AWQ-clip block 128,
11 clip ratios, 64 sampled tokens); MSE multiplier sweep (39 candidates) for INT8 per-channel,
INT4 block-128 and FP8 per-tensor amax.  CPU baseline (``--cpu``): the oracle on a row slice.
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
for p in (str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

VALU_PEAK = 256 * 4 * 64 / 2 * 2.4e9  # lane-instructions / s


def timed(fn, iters=20, warmup=3):
    s = torch.cuda.current_stream()
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()

    from modelopt_amd import _ext
    from modelopt_amd.torch.quantization.calib.mse import fp8_scale_candidates

    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    co, ci = 14336, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    w = (torch.randn(co, ci, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    res = {}

    # NVFP4 FP8-scale sweep (126 candidates / 16-element block)
    xb = w.view(-1, 16)
    ga = xb.float().abs().amax()
    cands = fp8_scale_candidates(dev)
    ms = timed(lambda: ops.nvfp4_fp8_scale_sweep(xb, ga, cands, 16), a.iters)
    n = w.numel()
    res["nvfp4_fp8_scale_sweep"] = {"shape": [co, ci], "candidates": 126, "ms": round(ms, 4),
                                    "G_elem_cand_per_s": round(n * 126 / ms / 1e6, 1),
                                    "weight_GB_s": round(n * 2 / ms / 1e6, 1)}

    # MSE multiplier sweep, 39 candidates
    mc = torch.linspace(0.25, 4.0, 39, device=dev)
    cases = {
        "mse_sweep_int8_per_channel": (w, w.float().abs().amax(1, keepdim=True).to(torch.bfloat16), 8),
        "mse_sweep_int4_block128": (w.view(-1, 128), w.view(-1, 128).float().abs().amax(1, keepdim=True), 4),
        "mse_sweep_fp8_per_tensor": (w.view(1, -1), w.float().abs().amax(), 0),
    }
    for name, (x, am, bits) in cases.items():
        ms = timed(lambda x=x, am=am, bits=bits: ops.mse_sweep(x, am, mc, bits, False, False, am.dim() != 0), a.iters)
        res[name] = {"shape": list(x.shape), "candidates": 39, "ms": round(ms, 4),
                     "G_elem_cand_per_s": round(n * 39 / ms / 1e6, 1)}

    # AWQ-clip: 64 tokens, block 128, 11 clip ratios (+ the original weight)
    ntok = 64
    xs = torch.randn(ntok, ci, device=dev, generator=g).to(torch.bfloat16).float().contiguous()
    wam = w.view(-1, 128).float().abs().amax(1, keepdim=True).to(torch.bfloat16)
    shr = torch.tensor([0.5, 0.55, 0.6, 0.65, 0.7, 0.75, 0.8, 0.85, 0.9, 0.95, 1.0])
    loss = torch.zeros(11, co, ci // 128, device=dev)
    ms = timed(lambda: ops.awq_clip_search(w, xs, wam, shr, loss, 128, 4, False, False, True), a.iters)
    macs = co * ci * 12 * ntok
    res["awq_clip_search"] = {"shape": [co, ci], "tokens": ntok, "variants": 12, "ms": round(ms, 4),
                              "TMAC_per_s": round(macs / ms / 1e9, 2)}

    if a.cpu:
        from oracle import ref_ops as R

        rows = 64
        t0 = time.perf_counter()
        R.nvfp4_fp8_scale_sweep(w[:rows].cpu(), ga.cpu(), 16)
        dt = time.perf_counter() - t0
        res["nvfp4_fp8_scale_sweep"]["cpu_oracle_G_elem_cand_per_s"] = round(rows * ci * 126 / dt / 1e9, 4)
        wc = w[:rows].cpu()
        t0 = time.perf_counter()
        R.awq_clip_block_losses(wc, xs.cpu().to(torch.bfloat16), wam[: rows * ci // 128].cpu(), shr.tolist(), 128)
        dt = time.perf_counter() - t0
        res["awq_clip_search"]["cpu_oracle_TMAC_per_s"] = round(rows * ci * 12 * ntok / dt / 1e12, 5)
        res["cpu_threads"] = torch.get_num_threads()
    print(json.dumps(res), flush=True)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
