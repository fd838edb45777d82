"""Diagnostic: where mtq_awq_scale_table differs from the CPU get_scale on this host, stage by
stage (torch CPU ops vs numpy's IEEE single-precision ops vs the GPU kernel)."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from modelopt_amd.torch.quantization import model_calib as MC  # noqa: E402

print("cpu capability", torch.backends.cpu.get_cpu_capability(), flush=True)
tiny = torch.finfo(torch.float32).tiny
I = lambda t: np.asarray(t, dtype=np.float32).view(np.int32)  # noqa: E731
for K in (33, 256):
    g = torch.Generator().manual_seed(K)
    x = (torch.rand(K, generator=g) * 12 - 6).exp2()
    w = torch.rand(K, generator=g) * 0.9 + 0.05
    x[::97] = 0.0
    for a in [k.item() for k in torch.arange(0, 1.1, 0.1)]:
        num, den = x.pow(a), w.pow(1 - a)
        q_t = num / (den + tiny)
        q_n = num.numpy() / (den.numpy() + np.float32(tiny))
        c_t = q_t.clamp(min=1e-4, max=1e4)
        c_n = np.minimum(np.maximum(q_n, np.float32(1e-4)), np.float32(1e4))
        p_t = c_t.max() * c_t.min()
        p_n = np.float32(c_n.max()) * np.float32(c_n.min())
        n_t = p_t.sqrt()
        n_n = np.sqrt(p_n)
        want_t = c_t / n_t
        want_n = c_n / n_n
        got = MC._scale_table(x.cuda(), w.cuda(), [a])[0].cpu().numpy()
        print(f"K {K} a {a:.3f}: q t/n {int((I(q_t) != I(q_n)).sum())} c {int((I(c_t) != I(c_n)).sum())} "
              f"p {float(p_t)!r}/{float(p_n)!r} n {float(n_t)!r}/{float(n_n)!r} "
              f"want t/n {int((I(want_t) != I(want_n)).sum())} got-vs-t {int((I(got) != I(want_t)).sum())} "
              f"got-vs-n {int((I(got) != I(want_n)).sum())} gpu max {float(got.max())!r}", flush=True)
