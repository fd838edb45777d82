#!/usr/bin/env python3
"""Cost of the AWQ weight-cache allocations (Llama-3-8B: per linear [11, N, K] bf16, 224 linears,
~154 GB): 224 separate torch.empty calls vs one slab of the same total, each followed by a write
of every byte (the cache fill), device synchronised; fresh caching allocator for each."""
import time

import torch

dev = torch.device("cuda")
shapes = []
for _ in range(32):
    shapes += [(4096, 4096), (1024, 4096), (1024, 4096), (4096, 4096), (14336, 4096), (14336, 4096), (4096, 14336)]
sizes = [11 * n * k * 2 for n, k in shapes]
total = sum(sizes)
torch.cuda.synchronize()


def run(label, f):
    torch.cuda.synchronize()
    t = time.perf_counter()
    bufs = f()
    torch.cuda.synchronize()
    ta = time.perf_counter() - t
    t = time.perf_counter()
    for b in bufs:
        b.fill_(1)
    torch.cuda.synchronize()
    tw = time.perf_counter() - t
    print(f"{label}: alloc {ta * 1e3:.1f} ms, first write {tw * 1e3:.1f} ms ({total / 1e9:.1f} GB)", flush=True)
    del bufs
    torch.cuda.empty_cache()


run("224 allocations", lambda: [torch.empty(s, dtype=torch.uint8, device=dev) for s in sizes])
run("one slab", lambda: [torch.empty(total, dtype=torch.uint8, device=dev)])
run("224 allocations again", lambda: [torch.empty(s, dtype=torch.uint8, device=dev) for s in sizes])
run("one slab again", lambda: [torch.empty(total, dtype=torch.uint8, device=dev)])
