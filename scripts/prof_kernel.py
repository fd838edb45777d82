#!/usr/bin/env python3
"""Drive one hot-path kernel for rocprofv3 (kernel trace / PMC passes).

Runs the bench.py dominant kernel (FP8 e4m3 static block-128 qdq, bf16 [32768, 4096]) `--iters`
times over 4 rotating 256 MiB inputs, so per-dispatch counters describe exactly the launch that
bench.py's roofline entry times.  `--kernel` selects another case of the suite.
"""

import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tensorrt-model-optimizer_amd"))

import torch  # noqa: E402

from modelopt_amd import _ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--kernel", default="fp8_block128")
args = ap.parse_args()

ops = _ext.ops()
T, H, B = 32768, 4096, 128
g = torch.Generator(device="cuda").manual_seed(1234)
xs = [torch.randn(T, H, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(4)]
blk = [x.view(-1, B).abs().amax(dim=1, keepdim=True).float() for x in xs]
amax = torch.tensor(8.0, device="cuda")
acc = torch.zeros(1, device="cuda")
hmax = torch.tensor([16.0 * 6], device="cuda")  # bench.py's histogram range
counts = torch.zeros(2048, dtype=torch.int32, device="cuda")
nv_bs = torch.ones(T, H // 16, device="cuda")  # bench.py's export_nvfp4_pack scales
i4_s = torch.full((T, H // 128), 0.01, device="cuda")  # bench.py's export_int4_pack scales
torch.cuda.synchronize()
for i in range(args.iters):
    x = xs[i % 4]
    if args.kernel == "fp8_block128":
        ops.quantize_op(x.view(-1, B), blk[i % 4], 8, 4, False, False)
    elif args.kernel == "fp8_per_tensor":
        ops.fake_e4m3fy(x, amax)
    elif args.kernel == "int8_per_tensor":
        ops.fake_tensor_quant(x, amax, 8, False, False)
    elif args.kernel == "mxfp4":
        ops.fused_amax_convert(x, 32, 6, 9, None)
    elif args.kernel == "hist":
        ops.histogram_abs_accumulate(x, hmax, counts, 2048, False)
    elif args.kernel == "nvfp4":
        ops.nvfp4_fake_quant_block(x, amax, 16)
    elif args.kernel == "amax":
        ops.amax_accumulate(x, acc, 1, 1, x.numel())
    elif args.kernel == "export_fp8":
        ops.export_fp8(x, amax / 448, False, True)
    elif args.kernel == "export_nvfp4":
        ops.export_nvfp4(x, nv_bs, amax / 2688)
    elif args.kernel == "export_int4":
        ops.export_int4(x, i4_s)
    elif args.kernel == "export_mxfp4":
        ops.export_mxfp4(x, 32)
    else:
        raise SystemExit(f"unknown kernel {args.kernel}")
torch.cuda.synchronize()
print("done", args.kernel, args.iters)
