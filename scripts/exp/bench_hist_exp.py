#!/usr/bin/env python3
"""A/B of the histogram experiment variants (scripts/exp/hist_exp.hip) against the product kernel,
bf16 [32768, 4096] (the bench.py input), 2048 bins, interleaved rounds in one process; every variant's
counts checked equal to the product's first (probe variant 4 excepted)."""
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
lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libhist_exp.so"))
lib.hist_exp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                         ctypes.c_void_p, ctypes.c_void_p]
VARS = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,4,40,41,44,45".split(","))]
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 7
MODE = sys.argv[3] if len(sys.argv) > 3 else "bench"
BIG = MODE.startswith("big") or MODE == "chunk"  # bench.py's 117 M-element input instead (big2: two of them, past the MALL)
NX = 2 if MODE == "big2" else 1 if MODE in ("big", "bench1", "chunk") else 4
g = torch.Generator(device="cuda").manual_seed(1234)
xs = []
for k in range(NX):
    if BIG:
        xs.append(torch.randn(8192, 14336, device="cuda", generator=torch.Generator(device="cuda").manual_seed(7 + k))
                  .to(torch.bfloat16))
        continue
    x = torch.randn(32768, 4096, device="cuda", dtype=torch.bfloat16, generator=g)
    cols = torch.randperm(4096, device="cuda", generator=g)[:4]
    x[:, cols] *= 16
    xs.append(x)
hmax = torch.tensor([16.0 * 6], device="cuda")
bins = 2048
stream = torch.cuda.current_stream().cuda_stream


def run_var(v, x, counts):
    rc = lib.hist_exp(v, x.data_ptr(), x.numel(), hmax.data_ptr(), bins, counts.data_ptr(), stream)
    assert rc == 0, rc


def run_prod(x, counts):
    ops.histogram_abs_accumulate(x, hmax, counts, bins, False)


ref = torch.zeros(bins, dtype=torch.int32, device="cuda")
run_prod(xs[0], ref)
for v in VARS:
    if v in (4, 44, 45, 114, 115):
        continue
    c = torch.zeros(bins, dtype=torch.int32, device="cuda")
    run_var(v, xs[0], c)
    torch.cuda.synchronize()
    assert torch.equal(c, ref), f"variant {v} counts differ"

arms = {"product": lambda x, c: run_prod(x, c)}
for v in VARS:
    arms[f"v{v}"] = (lambda vv: (lambda x, c: run_var(vv, x, c)))(v)
counts = torch.zeros(bins, dtype=torch.int32, device="cuda")
times = {k: [] for k in arms}
for _ in range(0 if MODE.startswith("chunk") else ROUNDS):
    for k, f in arms.items():
        for i in range(3):
            f(xs[i % len(xs)], counts)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(20):
            f(xs[i % len(xs)], counts)
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / 20)
if MODE.startswith("chunk"):
    # the chunked call: product (_histc_counts, 16 threads) vs the two experiment pairs
    from modelopt_amd.torch.quantization.calib.histogram import _histc_counts  # noqa: E402
    lib.hist_exp_chunked.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    scr = torch.zeros(256 * bins, dtype=torch.int32, device="cuda")
    hist = torch.zeros(bins, device="cuda")

    def pair(v):
        def f(x, c):
            assert lib.hist_exp_chunked(v, x.data_ptr(), x.numel(), hmax.data_ptr(), bins, scr.data_ptr(),
                                        hist.data_ptr(), stream) == 0
        return f
    ref = _histc_counts(xs[0], hmax, bins, False, threads=16)
    for v in (0, 1):
        pair(v)(xs[0], None)
        torch.cuda.synchronize()
        assert torch.equal(hist, ref), f"pair {v} differs"  # no count reaches 2^24 per chunk here
    arms = {"product_histc16": lambda x, c: _histc_counts(x, hmax, bins, False, threads=16),
            "pair_rows_atomic": pair(0), "pair_block_rows": pair(1)}
    times = {k: [] for k in arms}
    for _ in range(ROUNDS):
        for k, f in arms.items():
            for i in range(3):
                f(xs[i % len(xs)], None)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(20):
                f(xs[i % len(xs)], None)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20)
n = xs[0].numel()
out = {}
for k, t in times.items():
    ms = statistics.median(t)
    out[k] = {"us": round(ms * 1e3, 2), "min_us": round(min(t) * 1e3, 2),
              "frac": round(n * 2 / (ms * 1e-3) / 8e12, 4)}
out["input"] = ("bf16 [8192, 14336] randn" if BIG else "bf16 [32768, 4096] bench") + f" x{NX} rotating"
print(json.dumps(out))
