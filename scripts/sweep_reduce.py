#!/usr/bin/env python3
"""Sweep the launch variants of the non-per-tensor reductions (one process per variant):
per-column amax (MTQ_AMD_COLS_VARIANT), per-row / per-block amax (MTQ_AMD_ROWS_VARIANT) and the
2048-bin |x| histogram (MTQ_AMD_HIST_VARIANT), on Llama-3-8B calibration shapes, 4 rotating
buffers each.  Prints GB/s (algorithmic: one bf16 read) and us per launch; checks results."""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]

CHILD = r'''
import sys, json, torch
sys.path.insert(0, "%s/tensorrt-model-optimizer_amd"); sys.path.insert(0, "%s")
import bench
from modelopt_amd import _ext
ops = _ext.ops()
which = sys.argv[1]
out = {}
def mk(shape, seed=1):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.randn(*shape, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(4)]
def report(key, xs, ms):
    out[key] = [round(xs[0].numel() * 2 / (ms * 1e-3) / 1e9, 1), round(ms * 1e3, 2)]
if which == "cols":
    for shape in [(32768, 4096), (8192, 14336), (8192, 4096)]:
        xs = mk(shape)
        acc = torch.zeros(shape[1], device="cuda")
        fn = lambda x: ops.amax_accumulate(x, acc, x.shape[0], x.shape[1], 1) or acc
        _, ms = bench.time_kernel(fn, xs, 50, 10)
        want = torch.stack([x.abs().amax(0) for x in xs]).amax(0).float()
        assert torch.equal(acc, want), "cols mismatch"
        report("x".join(map(str, shape)), xs, ms)
elif which == "rows":
    for shape, q in [((32768, 4096), 4096), ((8192, 14336), 14336), ((32768, 4096), 128), ((14336, 4096), 128)]:
        xs = mk(shape)
        r = xs[0].numel() // q
        acc = torch.zeros(r, device="cuda")
        fn = lambda x: ops.amax_accumulate(x, acc, 1, r, q) or acc
        _, ms = bench.time_kernel(fn, xs, 50, 10)
        want = torch.stack([x.reshape(r, q).abs().amax(1) for x in xs]).amax(0).float()
        assert torch.equal(acc, want), "rows mismatch"
        report("x".join(map(str, shape)) + f"/q{q}", xs, ms)
else:
    for shape in [(32768, 4096), (8192, 14336)]:
        xs = mk(shape)
        for x in xs:
            x[:, :4] *= 16
        hmax = torch.tensor([max(float(x.abs().max()) for x in xs)], device="cuda")
        counts = torch.zeros(2048, dtype=torch.int32, device="cuda")
        fn = lambda x: ops.histogram_abs_accumulate(x, hmax, counts, 2048, False) or counts
        _, ms = bench.time_kernel(fn, xs, 50, 10)
        counts.zero_()
        ops.histogram_abs_accumulate(xs[0], hmax, counts, 2048, False)
        ref = torch.histc(xs[0].abs().float(), 2048, 0, float(hmax)).to(torch.int64).cpu()
        got = counts.to(torch.int64).cpu()
        assert int(got.sum()) == xs[0].numel(), "hist total"
        out["x".join(map(str, shape)) + "_l1_vs_torch_cuda"] = int((got - ref).abs().sum())
        report("x".join(map(str, shape)), xs, ms)
print(json.dumps(out))
''' % (REPO, REPO)

VARIANTS = {
    "cols": ("MTQ_AMD_COLS_VARIANT", {0: "wide auto", 1: "old per-lane slab", 5: "wide 1/CU", 3: "wide 2/CU", 4: "wide 0.5/CU"}),
    "rows": ("MTQ_AMD_ROWS_VARIANT", {0: "unrolled U=8 / short RU=4 (new)", 1: "old"}),
    "hist": ("MTQ_AMD_HIST_VARIANT", {0: "div rep4 2/CU", 8: "div rep8 1/CU", 9: "div rep8 2/CU", 1: "old"}),
}

res = {}
for which in sys.argv[1:] or list(VARIANTS):
    env_name, vs = VARIANTS[which]
    for v, label in vs.items():
        env = dict(os.environ, **{env_name: str(v)})
        r = subprocess.run([sys.executable, "-c", CHILD, which], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(which, v, r.stderr[-3000:])
            sys.exit(r.returncode)
        res.setdefault(which, {})[f"v{v} {label}"] = json.loads(r.stdout.strip().splitlines()[-1])
        print(which, v, label, res[which][f"v{v} {label}"], flush=True)
print(json.dumps(res, indent=1))
