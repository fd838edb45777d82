#!/usr/bin/env python3
"""One C5 phase per process for rocprofv3 kernel traces (Mixtral-8x7B dims, reduced depth): `bf16`
runs the calibration forward loop without quantizers, `calib` runs mtq.quantize(FP8_DEFAULT_CFG)
on the same loop -- the two traces' kernel totals split the quantizer overhead into GPU work and
host time.  python scripts/prof_c5_phase.py bf16|calib [layers] [samples]"""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from benchmarks import ptq_llama  # noqa: E402

phase = sys.argv[1]
layers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
samples = int(sys.argv[3]) if len(sys.argv) > 3 else 512
import modelopt_amd.torch.quantization as mtq  # noqa: E402

dev = torch.device("cuda")
ids = torch.randint(0, 32000, (samples, 512), device=dev, generator=torch.Generator(device=dev).manual_seed(1))
batches = list(ids.split(16))
model = ptq_llama.build_model(layers, dev, "mixtral-8x7b")
model.config._experts_implementation = "eager"


def loop(m):
    with torch.no_grad():
        for b in batches:
            m(b)


torch.cuda.synchronize()
t = time.perf_counter()
if phase == "bf16":
    loop(model)
else:
    mtq.quantize(model, mtq.FP8_DEFAULT_CFG, loop)
torch.cuda.synchronize()
print(phase, round(time.perf_counter() - t, 3), flush=True)
