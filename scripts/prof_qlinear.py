#!/usr/bin/env python3
"""Per-shape kernel durations of the decode QuantLinear kernels, for rocprofv3 --kernel-trace:
each Llama-3-8B linear shape runs `--iters` eager fused calls (INT4 block-128 and FP8 per-tensor)
at M = `--m`, shapes separated by device syncs, so the trace's kernels group by grid size.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ql -o ql -- python scripts/prof_qlinear.py
    python scripts/prof_qlinear.py --summarize gpurun_out/prof_ql/.../ql_kernel_trace.csv
"""
import argparse
import csv
import collections
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tensorrt-model-optimizer_amd"))

SHAPES = [(4096, 4096), (1024, 4096), (14336, 4096), (4096, 14336)]


def run(a):
    import torch
    from modelopt_amd import _ext

    ops = _ext.ops()
    g = torch.Generator(device="cuda").manual_seed(0)
    for n, k in SHAPES:
        w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16, generator=g) * 0.02
        x = torch.randn(a.m, k, device="cuda", dtype=torch.bfloat16, generator=g)
        a4 = w.float().reshape(-1, 128).abs().amax(1, keepdim=True)
        a8 = w.float().abs().amax().reshape(())
        for _ in range(a.iters):
            ops.qlinear_small_m(x, w, None, a4, 128, 0, 4, False, False)
        torch.cuda.synchronize()
        for _ in range(a.iters):
            ops.qlinear_small_m(x, w, None, a8, k, 1, 8, False, False)
        torch.cuda.synchronize()
    print("ok")


def summarize(path):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if "qlinear" not in name:
            continue
        kname = name.split("(")[0].split("::")[-1][:60]
        key = (kname, r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Workgroup_Size_X") or r.get("Workgroup_Size"))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for key, ds in sorted(agg.items(), key=lambda kv: -len(kv[1])):
        ds = sorted(ds)
        out[" ".join(map(str, key))] = {"n": len(ds), "median_us": round(ds[len(ds) // 2], 2), "min_us": round(ds[0], 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
    else:
        run(a)
