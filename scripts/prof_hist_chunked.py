#!/usr/bin/env python3
"""The histogram calibrator's >2^24-element call (bench.py ``histogram_2048_abs_117M_*``): bf16
[8192, 14336] (117.4 M elements, a Llama-3-8B down_proj input at batch 16), 2048 bins, torch.histc's
16-thread chunking.  Times, with HIP events on the launching stream, back to back:

* ``histc16``   -- the calibrator's ``_histc_counts(..., threads=16)`` (host logic + one launch);
* ``chunked``   -- ``ops.histogram_abs_chunked`` alone with the bounds / scratch prepared once;
* ``exact``     -- one exact-count launch over the same tensor (the roofline reference);
* ``histc16_skip`` -- ``skip_zeros=True`` (the compacted chunk bounds).

Run under ``rocprofv3 --kernel-trace --stats`` for the per-launch kernel durations.  Prints one JSON
line; the counts of ``chunked`` are checked equal to ``histc16``'s."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from modelopt_amd import _ext  # noqa: E402
from modelopt_amd.torch.quantization.calib import histogram as H  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ops = _ext.ops()
x = torch.randn(8192, 14336, device="cuda", generator=torch.Generator(device="cuda").manual_seed(7)).to(torch.bfloat16)
x.view(-1)[::97] = 0  # some zeros for the skip_zeros leg
hmax = torch.tensor([16.0 * 6], device="cuda")
counts = torch.zeros(2048, dtype=torch.int32, device="cuda")
n = x.numel()
threads = 16
chunk = -(-n // threads)
scratch = None  # the op's own (caching-allocator) rows
flat = x.view(-1)


def t(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w0 = time.perf_counter()
    s.record()
    for _ in range(ITERS):
        fn()
    e.record()
    w1 = time.perf_counter()
    torch.cuda.synchronize()
    return {"ms": round(s.elapsed_time(e) / ITERS, 4), "host_ms": round((w1 - w0) * 1e3 / ITERS, 4),
            "frac": round(n * 2 / (s.elapsed_time(e) / ITERS * 1e-3) / 8e12, 4)}


res = {
    "histc16": t(lambda: H._histc_counts(x, hmax, 2048, False, threads=16)),
    "chunked": t(lambda: ops.histogram_abs_chunked(flat, hmax, 2048, False, None, chunk, threads, scratch)),
    "exact": t(lambda: ops.histogram_abs_accumulate(x, hmax, counts, 2048, False)),
    "histc16_skip": t(lambda: H._histc_counts(x, hmax, 2048, True, threads=16)),
}
a = H._histc_counts(x, hmax, 2048, False, threads=16)
b = ops.histogram_abs_chunked(flat, hmax, 2048, False, None, chunk, threads, scratch)
res["chunked_equals_histc16"] = bool(torch.equal(a, b))
res["elements"] = n
print(json.dumps(res))
