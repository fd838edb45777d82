#!/usr/bin/env python3
"""Measurement only: workgroup-size A/B of the dynamic NVFP4 qdq kernel (scripts/exp/tpb_exp.hip) on
the bench.py input (4 rotating bf16 [32768, 4096]), interleaved rounds of 50 launches; every variant's
output equals the product op's bit for bit."""
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
lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libtpb_exp.so"))
lib.tpb_exp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                        ctypes.c_void_p]
ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 11
g = torch.Generator(device="cuda").manual_seed(1234)
xs = []
for _ in range(4):
    x = torch.randn(32768, 4096, device="cuda", dtype=torch.bfloat16, generator=g)
    cols = torch.randperm(4096, device="cuda", generator=g)[:4]
    x[:, cols] *= 16
    xs.append(x)
amax_t = torch.tensor(8.0, device="cuda")
y = torch.empty_like(xs[0])
stream = torch.cuda.current_stream().cuda_stream
n = xs[0].numel()


def var(v):
    def f(i):
        assert lib.tpb_exp(v, xs[i].data_ptr(), y.data_ptr(), n, amax_t.data_ptr(), stream) == 0
    return f


ref = ops.nvfp4_fake_quant_block(xs[0], amax_t, 16)
for v in (256, 512, 1024):
    var(v)(0)
    torch.cuda.synchronize()
    assert torch.equal(y, ref), v
arms = {f"tpb{v}": var(v) for v in (256, 512, 1024)}
arms["product_op"] = lambda i: ops.nvfp4_fake_quant_block(xs[i], amax_t, 16)
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
print(json.dumps({k: {"us": round(statistics.median(v) * 1e3, 2), "frac": round(n * 4 / (statistics.median(v) * 1e-3) / 8e12, 4)}
                  for k, v in t.items()}))
