"""Error statistics of mtq_attention_fwd vs the reference goldens (tests/golden/attention.*)."""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO), str(REPO / "tests")]
import torch  # noqa: E402
from safetensors.torch import load_file  # noqa: E402

from modelopt_amd.torch.kernels.common.attention import attention  # noqa: E402
from test_gpu_attention import META, _kw  # noqa: E402

g = load_file(str(REPO / "tests/golden/attention.safetensors"))
out = {}
for name, mt in sorted(META.items()):
    q, k, v = (g[f"{name}.{t}"].cuda() for t in "qkv")
    o = attention(q, k, v, **_kw(mt, "cuda")).cpu()
    s = max(mt["lens_q"])
    valid = torch.zeros(q.shape[0], dtype=torch.bool)
    for i, n in enumerate(mt["lens_q"]):
        valid[i * s: i * s + n] = True
    o = torch.where(valid[:, None, None], o, torch.zeros((), dtype=o.dtype)).float()
    w = g[f"{name}.o"].float()
    e = (o - w).abs()
    ulp = torch.finfo(g[f"{name}.o"].dtype).eps * torch.maximum(w.abs(), torch.tensor(2.0 ** -6))
    out[name] = {"max_abs": float(e.max()), "mean_abs": float(e.mean()), "max_ulp": float((e / ulp).max()),
                 "frac_exact": float((e == 0).float().mean()), "frac_le_1ulp": float((e <= ulp).float().mean())}
print(json.dumps(out, indent=1))
