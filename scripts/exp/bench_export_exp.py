#!/usr/bin/env python3
"""Measurement only: MXFP4 export packer variants (scripts/exp/export_exp.hip) against the product
op on the bench.py input ([32768, 4096] bf16, 4 rotating 256 MiB buffers), interleaved rounds;
every variant's codes and scale bytes must equal the product's bit for bit.  Fraction of the 8 TB/s
roofline at 2.5 B per element (bench.py's accounting for export_mxfp4_pack)."""
import ctypes
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from modelopt_amd import _ext  # noqa: E402

ops = _ext.ops()
lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libexport_exp.so"))
lib.export_exp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
VARS = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "5,6,7,8,9,10".split(","))]
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 7
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
xs = []
for _ in range(4):
    x = torch.randn(32768, 4096, device=dev, generator=g).to(torch.bfloat16)
    x[:, ::1000] *= 16
    xs.append(x)
n = xs[0].numel()
stream = torch.cuda.current_stream().cuda_stream
ys = torch.empty(n // 2, dtype=torch.uint8, device=dev)
ss = torch.empty(n // 32, dtype=torch.uint8, device=dev)


def product(x):
    return ops.export_mxfp4(x, 32)


def var(v):
    def f(x):
        rc = lib.export_exp(v, x.data_ptr(), ys.data_ptr(), ss.data_ptr(), n, stream)
        assert rc == 0, rc
    return f


for v in VARS:
    if v == 15:  # probe: output deliberately wrong
        continue
    for x in xs[:2]:
        yp, sp = product(x)
        ys.fill_(0x5A)
        ss.fill_(0x5A)
        var(v)(x)
        torch.cuda.synchronize()
        assert torch.equal(ys, yp.reshape(-1)) and torch.equal(ss, sp.reshape(-1)), v
arms = {"product": product}
arms.update({f"v{v}": var(v) for v in VARS})
t = {k: [] for k in arms}
steps = 40
for _ in range(ROUNDS):
    for k, f in arms.items():
        for i in range(4):
            f(xs[i])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(steps):
            f(xs[i % 4])
        e1.record()
        torch.cuda.synchronize()
        t[k].append(e0.elapsed_time(e1) / steps)
res = {}
for k, v in t.items():
    ms = statistics.median(v)
    res[k] = {"ms": round(ms, 4), "min_ms": round(min(v), 4), "frac": round(n * 2.5 / (ms * 1e-3) / 8e12, 4)}
print(json.dumps(res))
