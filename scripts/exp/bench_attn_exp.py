#!/usr/bin/env python3
"""Per-wave time split of the fused attention kernel (scripts/exp/attn_exp.hip = csrc/mtq_attention.hip
plus s_memtime stamps) at the bench shape (16 x 512, 32 / 8 heads, D 128, bf16, causal): per pass
(long tile, short tile) the prologue (Q + first K/V stage landed), the stage loop and the epilogue,
in shader cycles, beside the launch time without stamps.  Output checked equal to the product's.
    python scripts/exp/bench_attn_exp.py [none|fp8] [out.json]"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
import torch  # noqa: E402

from modelopt_amd.torch.kernels.common.attention import attention  # noqa: E402

lib = ctypes.CDLL(str(REPO / "scripts/exp/libattn_exp.so"))
lib.attn_exp_set_stamps.argtypes = [ctypes.c_void_p]
lib.attn_exp_fwd.argtypes = [ctypes.c_void_p] * 8 + [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
                                                                         ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
mode = sys.argv[1] if len(sys.argv) > 1 else "none"
out_path = sys.argv[2] if len(sys.argv) > 2 else None
dev = torch.device("cuda")
B, S, HQ, HKV, D = 16, 512, 32, 8, 128
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B * S, HQ, D, device=dev, generator=g).bfloat16()
k = torch.randn(B * S, HKV, D, device=dev, generator=g).bfloat16()
v = torch.randn(B * S, HKV, D, device=dev, generator=g).bfloat16()
start = (torch.arange(B, device=dev) * S).int()
lens = torch.full((B,), S, device=dev, dtype=torch.int32)
o = torch.empty_like(q)
strides = (ctypes.c_int64 * 12)(*([0, HQ * D, D] + [0, HKV * D, D] * 2 + [0, HQ * D, D]))
pm, ps = (0, 0.0) if mode == "none" else (1, 1.0 / 448.0)
stream = torch.cuda.current_stream().cuda_stream
ref = attention(q, k, v, start, lens, S, p_qdq=None if mode == "none" else mode)


def launch():
    rc = lib.attn_exp_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), start.data_ptr(), lens.data_ptr(),
                          start.data_ptr(), lens.data_ptr(), B, S, HQ, HKV, D, strides, 1, D ** -0.5, pm, ps, 2, stream)
    assert rc == 0, rc


def timed(iters=50):
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


res = {"mode": mode}
assert lib.attn_exp_set_stamps(None) == 0


res["ms_no_stamps"] = timed()
# (A/B of versions: scripts/exp/bench_attn_ab.py -- rotated order; a fixed order biases ~4 %)
launch()
torch.cuda.synchronize()
res["equal_to_product"] = bool(torch.equal(o, ref))
nwg = 2 * HQ * B  # one pair of query tiles per workgroup
st = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device=dev)
assert lib.attn_exp_set_stamps(st.data_ptr()) == 0
res["ms_stamps"] = timed(10)
st.zero_()
launch()
torch.cuda.synchronize()
assert lib.attn_exp_set_stamps(None) == 0
t = st.view(nwg, 4, 8).double()
t0 = t[..., 0].min()
res["kernel_cycles"] = float(t[..., 7].max() - t0)
seg = {"p0_prologue": (0, 1), "p0_loop": (1, 2), "p0_epilogue": (2, 3), "between": (3, 4),
       "p1_prologue": (4, 5), "p1_loop": (5, 6), "p1_epilogue": (6, 7)}
for name, (i, j) in seg.items():
    d = (t[..., j] - t[..., i]).flatten()
    res[name] = {"mean": float(d.mean()), "p10": float(d.quantile(0.1)), "p90": float(d.quantile(0.9))}
life = (t[..., 7] - t[..., 0]).flatten()
res["wave_life"] = {"mean": float(life.mean()), "p10": float(life.quantile(0.1)), "p90": float(life.quantile(0.9))}
starts = (t[:, 0, 0] - t0)
res["wg_start_quantiles"] = [float(starts.quantile(x)) for x in (0.0, 0.25, 0.5, 0.75, 1.0)]
print(json.dumps(res, indent=1))
if out_path:
    Path(out_path).write_text(json.dumps(res, indent=1))
