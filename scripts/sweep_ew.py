#!/usr/bin/env python3
"""Time the element-wise fake-quant kernels under each MTQ_AMD_EW_VARIANT launch structure
(`--env MTQ_AMD_GROUP_VARIANT --variants 0,1` sweeps another launch knob instead).

Each variant runs in its own process (the variant is read once per process); all variants run
interleaved rounds so device-clock drift hits them equally (cdna_hip_programming.md §5.4 rule 24).
"""
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
xs = bench.make_inputs(1234)
blk = [x.view(-1, 128).abs().amax(dim=1, keepdim=True).float() for x in xs]
idx = {id(x): i for i, x in enumerate(xs)}
a = torch.tensor(8.0, device="cuda")
cases = {
  "fp8_block128": lambda x: ops.quantize_op(x.view(-1, 128), blk[idx[id(x)]], 8, 4, False, False),
  "fp8_tensor": lambda x: ops.fake_e4m3fy(x, a),
  "int8_tensor": lambda x: ops.fake_tensor_quant(x, a, 8, False, False),
  "int4_block128": lambda x: ops.quantize_op(x.view(-1, 128), blk[idx[id(x)]], 4, 0, False, False),
  "fp8_block128_bf16amax": lambda x: ops.quantize_op(x.view(-1, 128), blkb[idx[id(x)]], 8, 4, False, False),
}
blkb = [b.to(torch.bfloat16) for b in blk]
out = {}
n = xs[0].numel()
for k, fn in cases.items():
    _, ms = bench.time_kernel(fn, xs, 50, 10)
    out[k] = round(n * 4 / (ms * 1e-3) / 1e9, 1)
print(json.dumps(out))
''' % (REPO, REPO)

ENV = sys.argv[sys.argv.index("--env") + 1] if "--env" in sys.argv else "MTQ_AMD_EW_VARIANT"
VARS = [int(v) for v in sys.argv[sys.argv.index("--variants") + 1].split(",")] if "--variants" in sys.argv else list(range(5))
res = {}
for rnd in range(2):
    for v in VARS:
        env = dict(os.environ, **{ENV: str(v)})
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            sys.exit(r.returncode)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        for k, val in d.items():
            res.setdefault(f"v{v}", {}).setdefault(k, []).append(val)
print(ENV, json.dumps(res, indent=1))
