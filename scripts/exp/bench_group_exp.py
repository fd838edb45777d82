#!/usr/bin/env python3
"""Measurement only: A/B of the FP8 static block-128 group kernel variants (scripts/exp/group_exp.hip)
on the bench.py primary input (4 rotating bf16 [32768, 4096], per-block fp32 amax), interleaved
rounds of 50 launches; both variants' outputs equal the product op's bit for bit."""
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
lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libgroup_exp.so"))
lib.group_exp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                          ctypes.c_void_p]
ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 9
g = torch.Generator(device="cuda").manual_seed(1234)
xs, am = [], []
for _ in range(4):
    x = torch.randn(32768, 4096, device="cuda", dtype=torch.bfloat16, generator=g)
    cols = torch.randperm(4096, device="cuda", generator=g)[:4]
    x[:, cols] *= 16
    xs.append(x)
    am.append(x.view(-1, 128).abs().amax(dim=1, keepdim=True).float())
y = torch.empty_like(xs[0])
stream = torch.cuda.current_stream().cuda_stream
n = xs[0].numel()


def var(v):
    def f(i):
        assert lib.group_exp(v, xs[i].data_ptr(), y.data_ptr(), n, am[i].data_ptr(), stream) == 0
    return f


def prod(i):
    return ops.quantize_op(xs[i].view(-1, 128), am[i], 8, 4, False, False)


ref = prod(0).view(-1)
for v in (0, 1, 2, 3, 4):
    var(v)(0)
    torch.cuda.synchronize()
    assert torch.equal(y.view(-1), ref), v
arms = {"v0_product": var(0), "v1_clamped": var(1), "v2_tpb512": var(2), "v3_tpb1024": var(3), "v4_tpb256": var(4), "product_op": lambda i: prod(i)}
t = {k: [] for k in arms}
for _ in range(ROUNDS):
    for k, f in arms.items():
        for i in range(4):
            f(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(50):
            f(i % 4)
        e1.record()
        torch.cuda.synchronize()
        t[k].append(e0.elapsed_time(e1) / 50)
res = {k: {"us": round(statistics.median(v) * 1e3, 2), "min_us": round(min(v) * 1e3, 2),
           "frac": round((n * 4 + n // 128 * 4) / (statistics.median(v) * 1e-3) / 8e12, 4)} for k, v in t.items()}
print(json.dumps(res))
