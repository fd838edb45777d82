#!/usr/bin/env python3
"""Measurement only: the FP8 per-tensor and NVFP4 export packers at U = 4 / 2 vectors per lane
(scripts/exp/export_exp.hip export_exp2) against the product ops on bench.py's input ([32768, 4096]
bf16, 4 rotating buffers), interleaved rounds; codes must equal the product's bit for bit.
Fractions of 8 TB/s at bench.py's accounting (3 B / element FP8, 2.5 B / element NVFP4)."""
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
lib = ctypes.CDLL(str(REPO / "scripts/exp/libexport_exp.so"))
lib.export_exp2.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 7
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
R, C = 32768, 4096
xs = [torch.randn(R, C, device=dev, generator=g).to(torch.bfloat16) for _ in range(4)]
n = R * C
stream = torch.cuda.current_stream().cuda_stream
amax_t = torch.tensor(8.0, device=dev)
s8 = (amax_t / 448).reshape(1)
nv_bs = torch.ones(n // 16, device=dev)
s2 = (amax_t / 2688).reshape(1)
y8 = torch.empty(n, dtype=torch.uint8, device=dev)
y4 = torch.empty(n // 2, dtype=torch.uint8, device=dev)


def var(v):
    y, a0, a1 = (y8, s8, s8) if v in (20, 21) else (y4, nv_bs, s2)

    def f(x):
        rc = lib.export_exp2(v, x.data_ptr(), y.data_ptr(), a0.data_ptr(), a1.data_ptr(), R, C, stream)
        assert rc == 0, rc
    return f


arms = {
    "fp8_product": (lambda x: ops.export_fp8(x, amax_t / 448, False, True), 3.0),
    "fp8_u4": (var(20), 3.0), "fp8_u2": (var(21), 3.0),
    "nvfp4_product": (lambda x: ops.export_nvfp4(x, nv_bs, amax_t / 2688), 2.5),
    "nvfp4_u4": (var(22), 2.5), "nvfp4_u2": (var(23), 2.5),
}
for v, ref, y in ((20, "fp8_product", y8), (21, "fp8_product", y8), (22, "nvfp4_product", y4), (23, "nvfp4_product", y4)):
    yp = arms[ref][0](xs[0])
    y.fill_(0x5A)
    var(v)(xs[0])
    torch.cuda.synchronize()
    assert torch.equal(y, yp.reshape(-1).view(torch.uint8)), v
t = {k: [] for k in arms}
steps = 40
for _ in range(ROUNDS):
    for k, (f, _) in arms.items():
        f(xs[0])
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
    res[k] = {"ms": round(ms, 4), "frac": round(n * arms[k][1] / (ms * 1e-3) / 8e12, 4)}
print(json.dumps(res))
