#!/usr/bin/env python3
"""One-shot check of the call the AWQ wide-linear path avoids: torch.bmm of
the pre-scaled activations [G, M, K] with the transposed view of the per-alpha weights [G, N, K]
-> [G, K, N] (strides (N*K, 1, K)), against per-slice torch.mm into one [G, M, N] buffer (what the
product runs).  Each step synchronised and printed before the next, shapes in increasing output
size; bit-equality of the two results is reported."""
import sys

import torch

dev = torch.device("cuda")
G, M = 11, 8192
for N, K in ((4096, 4096), (14336, 4096)):
    gen = torch.Generator(device=dev).manual_seed(N)
    xs = torch.randn(G, M, K, device=dev, generator=gen, dtype=torch.bfloat16)
    wq = (torch.randn(G, N, K, device=dev, generator=gen, dtype=torch.bfloat16) * 0.02)
    wt = wq.transpose(1, 2)
    print(f"[{G},{M},{K}] x [{G},{K},{N}] strides {tuple(wt.stride())} out {G * M * N * 2 / 2**20:.0f} MiB "
          f"ptr%256 x {xs.data_ptr() % 256} w {wq.data_ptr() % 256}", flush=True)
    ref = torch.empty(G, M, N, device=dev, dtype=torch.bfloat16)
    for g in range(G):
        torch.mm(xs[g], wq[g].t(), out=ref[g])
    torch.cuda.synchronize()
    print("  per-slice mm ok", flush=True)
    out = torch.bmm(xs, wt)
    torch.cuda.synchronize()
    print("  bmm ok; bit-equal to per-slice mm:", bool(torch.equal(out, ref)),
          "max abs diff", (out.float() - ref.float()).abs().max().item(), flush=True)
    del xs, wq, wt, ref, out
    torch.cuda.empty_cache()
sys.exit(0)
