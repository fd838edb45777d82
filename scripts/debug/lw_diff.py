import sys
sys.path.insert(0, "tensorrt-model-optimizer_amd"); sys.path.insert(0, ".")
import torch
from safetensors.torch import load_file
import modelopt_amd.torch.quantization as mtq
from tests.test_gpu_mtq import _tiny_llama, G

t = load_file(str(G / "llama_fp8.safetensors"))
want = {k[5:]: v for k, v in t.items() if k.startswith("amax.")}
for use_cache in (True, False):
    for lw in (False, True):
        model = _tiny_llama()
        model.load_state_dict({k[3:]: v for k, v in t.items() if k.startswith("sd.")})
        model.config.use_cache = use_cache
        model.to("cuda")
        ids = t["calib_ids"].to("cuda")
        cfg = {**mtq.FP8_DEFAULT_CFG, "algorithm": {"method": "max", "layerwise": {"enable": lw}}}
        mtq.quantize(model, cfg, lambda mm: [mm(b) for b in ids])
        for n, q in model.named_modules():
            if isinstance(q, mtq.TensorQuantizer) and q.amax is not None and n in want:
                a, b = float(q.amax), float(want[n])
                if abs(a - b) > 1e-5 * abs(b):
                    print(f"cache={use_cache} lw={lw} {n}: got {a:.6g} want {b:.6g}")
print("done")
