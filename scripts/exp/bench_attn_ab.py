#!/usr/bin/env python3
"""Fair A/B/C of fused-attention kernel versions: copies built by scripts/exp/mk_attn_exp.py (REV
NAME -> libNAME.so, all called through ctypes the same way) at the bench shape (16 x 512, 32 / 8
heads, D 128, bf16, causal), timed with HIP events in rounds whose order rotates (a fixed order
biased the later arm by ~4 %), outputs checked bit-equal across versions.
    python scripts/exp/bench_attn_ab.py none|fp8 name1,name2,... [rounds] [out.json]"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[2]
mode = sys.argv[1]
names = sys.argv[2].split(",")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 12
out_path = sys.argv[4] if len(sys.argv) > 4 else None
dev = torch.device("cuda")
B, S, HQ, HKV, D = 16, 512, 32, 8, 128
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B * S, HQ, D, device=dev, generator=g).bfloat16()
k = torch.randn(B * S, HKV, D, device=dev, generator=g).bfloat16()
v = torch.randn(B * S, HKV, D, device=dev, generator=g).bfloat16()
start = (torch.arange(B, device=dev) * S).int()
lens = torch.full((B,), S, device=dev, dtype=torch.int32)
strides = (ctypes.c_int64 * 12)(*([0, HQ * D, D] + [0, HKV * D, D] * 2 + [0, HQ * D, D]))
pm, ps = (0, 0.0) if mode == "none" else (1, 1.0 / 448.0)
stream = torch.cuda.current_stream().cuda_stream
fns, outs = {}, {}
for n in names:
    lib = ctypes.CDLL(str(REPO / f"scripts/exp/lib{n}.so"))
    f = getattr(lib, f"{n}_fwd")
    f.argtypes = [ctypes.c_void_p] * 8 + [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
                                                              ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
    assert getattr(lib, f"{n}_set_stamps")(None) == 0
    o = torch.empty_like(q)

    def launch(f=f, o=o):
        rc = f(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), start.data_ptr(), lens.data_ptr(),
               start.data_ptr(), lens.data_ptr(), B, S, HQ, HKV, D, strides, 1, D ** -0.5, pm, ps, 2, stream)
        assert rc == 0, rc
    fns[n], outs[n] = launch, o


def timed(fn, iters=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


ms = {n: [] for n in names}
for r in range(rounds):
    order = names[r % len(names):] + names[:r % len(names)]
    for n in order:
        ms[n].append(timed(fns[n]))
res = {"mode": mode, "rounds": rounds, "ms_median": {n: statistics.median(v) for n, v in ms.items()},
       "ms_all": ms}
for n in names:
    fns[n]()
torch.cuda.synchronize()
res["equal_to_first"] = {n: bool(torch.equal(outs[n], outs[names[0]])) for n in names}
print(json.dumps({k: v for k, v in res.items() if k != "ms_all"}, indent=1))
if out_path:
    Path(out_path).write_text(json.dumps(res, indent=1))
