#!/usr/bin/env python3
"""How long the AWQ search's quantised-weight cache allocation takes on the box: one 150 GB
torch.empty versus the 224 per-linear allocations of the C3 cache (Llama-3-8B: 32 layers x
{q, o: 11 x 4096 x 4096, k, v: 11 x 1024 x 4096, gate, up: 11 x 14336 x 4096, down: 11 x 4096 x
14336} bf16), each followed by a first write; host wall-clock per phase."""
import json
import time

import torch

dev = torch.device("cuda")
torch.cuda.synchronize()
res = {}
shapes = [(4096, 4096), (1024, 4096), (1024, 4096), (4096, 4096), (14336, 4096), (14336, 4096), (4096, 14336)] * 32
t0 = time.perf_counter()
bufs = [torch.empty((11, n, k), dtype=torch.bfloat16, device=dev) for n, k in shapes]
t1 = time.perf_counter()
for b in bufs:
    b.fill_(1)
torch.cuda.synchronize()
t2 = time.perf_counter()
for b in bufs:
    b.fill_(2)
torch.cuda.synchronize()
t3 = time.perf_counter()
total = sum(b.numel() * 2 for b in bufs)
res["per_linear"] = {"n": len(bufs), "gb": round(total / 1e9, 1), "alloc_s": round(t1 - t0, 3),
                     "first_fill_s": round(t2 - t1, 3), "second_fill_s": round(t3 - t2, 3)}
del bufs, b
torch.cuda.empty_cache()
torch.cuda.synchronize()
t0 = time.perf_counter()
one = torch.empty(total, dtype=torch.uint8, device=dev)
t1 = time.perf_counter()
one.fill_(1)
torch.cuda.synchronize()
t2 = time.perf_counter()
one.fill_(2)
torch.cuda.synchronize()
t3 = time.perf_counter()
res["one_block"] = {"alloc_s": round(t1 - t0, 3), "first_fill_s": round(t2 - t1, 3), "second_fill_s": round(t3 - t2, 3)}
del one
torch.cuda.empty_cache()
print(json.dumps(res))
