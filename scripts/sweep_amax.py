#!/usr/bin/env python3
"""Time the per-tensor amax reduction under each MTQ_AMD_AMAX_VARIANT (one process per variant,
interleaved rounds) at the calibration shapes: Llama-3-8B activations per batch of 16x512 tokens
([8192, 4096], [8192, 14336]) and the bench's [32768, 4096]; 4 rotating buffers each."""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]

CHILD = r'''
import sys, json, torch
sys.path.insert(0, "%s/tensorrt-model-optimizer_amd"); sys.path.insert(0, "%s")
import bench
from modelopt_amd import _ext
ops = _ext.ops()
out = {}
acc = torch.zeros(1, device="cuda")
for shape in [(8192, 4096), (8192, 14336), (32768, 4096), (14336, 4096)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(*shape, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(4)]
    want = max(float(x.abs().max()) for x in xs)
    def fn(x):
        ops.amax_accumulate(x, acc, 1, 1, x.numel())
        return acc
    _, ms = bench.time_kernel(fn, xs, 50, 10)
    assert float(acc) == want, (float(acc), want)
    acc.zero_()
    out["x".join(map(str, shape))] = [round(xs[0].numel() * 2 / (ms * 1e-3) / 1e9, 1), round(ms * 1e3, 2)]
print(json.dumps(out))
''' % (REPO, REPO)

res = {}
for rnd in range(2):
    for v in range(5):
        env = dict(os.environ, MTQ_AMD_AMAX_VARIANT=str(v))
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            sys.exit(r.returncode)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        for k, val in d.items():
            res.setdefault(f"v{v}", {}).setdefault(k, []).append(val)
print("GB/s, us per launch; v0 persistent 1024 thr U=8 2 blk/CU (default), v1 grid-stride 256 thr, v2 U=8 1 blk/CU, v3 U=8 4 blk/CU, v4 U=4 2 blk/CU")
print(json.dumps(res, indent=1))
