#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE on the CPU.

Run in the survey container only (it needs /root/reference; the GPU box never runs this):

    python tests/golden/make_golden.py

How the reference is imported: the reference package is importable from /root/reference with
three tiny import shims created under /tmp/mo_shim (outside both repositories): a
``nvidia_modelopt-0.0.0.dist-info/METADATA`` so ``modelopt/__init__.py`` can read its version, and
stub ``omegaconf`` / ``pulp`` modules that the reference imports at module load for features off
the fake-quant path (robust_json, the LP searcher).  None of the code under test is stubbed.

Outputs (small; committed):
  tensor_quant.safetensors   INT `_tensor_quant`, FP8 `fp8_eager`, `reduce_amax` cases
  quantizer.safetensors      TensorQuantizer calibrate+quant cases (per-tensor, axis, block, padding)
  calib.safetensors/.json    MaxCalibrator / HistogramCalibrator (+ entropy / percentile amax)
  calib_ref.safetensors/.json HistogramCalibrator at > 2^24 counts per call (1 / 3 threads) + MSE amax
  mtq_linear.safetensors     C1: mtq.quantize(nn.Linear(1024,1024), INT8_DEFAULT_CFG)
  llama_fp8.safetensors      C2 class: tiny LlamaForCausalLM FP8_DEFAULT_CFG PTQ (amax + logits)
  awq.safetensors/.json      C3 class: awq_lite on a small MLP (best alpha/scale, weights, amax)
  awq_b128.safetensors/.json C3 proper: INT4_AWQ_CFG (block 128) in bf16 on K % 128 == 0 linears
  prod.safetensors/.json     E2E at production shapes: 2-layer Llama-3-8B-shaped FP8 / INT8 / INT4-AWQ
                             and a hidden-1024 8-expert Mixtral layer FP8 (amax, AWQ scales, logits;
                             weights regenerated from the seed, pinned by sha256)
  presets.json               the reference preset configs
  mx_kat.json                the MX known-answer tables of test_quantize_mxformats_cuda.py (data)
"""

from __future__ import annotations

import ast
import json
import os
import sys
from pathlib import Path

OUT = Path(__file__).resolve().parent
REF = Path(os.environ.get("MTQ_REFERENCE", "/root/reference"))
SHIM = Path("/tmp/mo_shim")


def _make_shim():
    (SHIM / "nvidia_modelopt-0.0.0.dist-info").mkdir(parents=True, exist_ok=True)
    (SHIM / "nvidia_modelopt-0.0.0.dist-info" / "METADATA").write_text(
        "Metadata-Version: 2.1\nName: nvidia-modelopt\nVersion: 0.0.0\n"
    )
    (SHIM / "omegaconf").mkdir(exist_ok=True)
    (SHIM / "omegaconf" / "__init__.py").write_text(
        "class DictConfig(dict): pass\nclass ListConfig(list): pass\n"
        "class OmegaConf:\n    @staticmethod\n    def to_container(x, *a, **k): return x\n"
        "    @staticmethod\n    def create(x=None, *a, **k): return x\n"
    )
    (SHIM / "pulp").mkdir(exist_ok=True)
    (SHIM / "pulp" / "__init__.py").write_text(
        "class _Dummy:\n    def __init__(self, *a, **k): pass\ndef __getattr__(name): return _Dummy\n"
    )
    sys.path[:0] = [str(SHIM), str(REF)]
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True


_make_shim()

# the reference's Triton kernels (NVFP4 golden) run on CPU through the Triton interpreter; it
# must be selected before any @triton.jit decoration happens
os.environ.setdefault("TRITON_INTERPRET", "1")

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
from safetensors.torch import save_file as _save_file  # noqa: E402

import modelopt.torch.quantization as mtq  # noqa: E402
from modelopt.torch.quantization import tensor_quant as tq  # noqa: E402
from modelopt.torch.quantization.calib import HistogramCalibrator, MaxCalibrator  # noqa: E402
from modelopt.torch.quantization.config import QuantizerAttributeConfig  # noqa: E402
from modelopt.torch.quantization.nn import TensorQuantizer  # noqa: E402
from modelopt.torch.quantization.utils import reduce_amax  # noqa: E402

torch.set_num_threads(8)


def save_file(t, path):
    _save_file({k: v.detach().clone().contiguous() for k, v in t.items()}, path)


def edges(shape, dtype, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(shape, generator=g) * scale
    f = x.view(-1)
    k = max(1, f.numel() // 64)
    f[:k] = torch.round(f[:k] * 8) / 8 + 0.5 / 8
    f[k : 2 * k] = 0.0
    f[2 * k : 3 * k] = -0.0
    f[3 * k] = 7.5 * scale
    return x.to(dtype)


DT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}


def gen_tensor_quant():
    t, meta = {}, []
    for dn, dt in DT.items():
        x = edges((64, 136), dt, seed=1)
        g = torch.Generator().manual_seed(2)
        amaxes = {
            "tensor": torch.tensor(2.5),
            "row": torch.rand(64, 1, generator=g) * 3 + 0.05,
            "col": torch.rand(1, 136, generator=g) * 3 + 0.05,
        }
        amaxes["row"][3] = 0.0
        amaxes["col"][0, 5] = 1e-30
        t[f"x_{dn}"] = x.clone()
        for an, a in amaxes.items():
            t[f"amax_{dn}_{an}"] = a.clone()
            for nb, u, nr in [(8, False, True), (8, False, False), (4, False, False), (4, True, False), (3, False, True)]:
                xi = x.abs() if u else x
                key = f"int_{dn}_{an}_b{nb}_u{int(u)}_n{int(nr)}"
                t[key + "_y"] = tq._tensor_quant(xi, a, nb, u, nr).contiguous()
                meta.append({"key": key, "x": f"x_{dn}", "abs": u, "amax": f"amax_{dn}_{an}",
                             "num_bits": nb, "unsigned": u, "narrow_range": nr})
            key = f"fp8_{dn}_{an}"
            t[key + "_y"] = tq.fp8_eager(x * 3, a).contiguous()
            meta.append({"key": key, "x": f"x_{dn}", "x_scale": 3.0, "amax": f"amax_{dn}_{an}", "fp8": True})
        # block-128 view, FP8 and INT4
        xb = edges((32, 256), dt, seed=3).view(-1, 128)
        ab = xb.float().abs().amax(dim=1, keepdim=True)
        t[f"blk_{dn}_x"], t[f"blk_{dn}_amax"] = xb.clone(), ab.clone()
        t[f"fp8blk_{dn}_y"] = tq.fp8_eager(xb, ab).contiguous()
        t[f"int4blk_{dn}_y"] = tq._tensor_quant(xb, ab, 4, False, False).contiguous()
        # plain e4m3 cast (amax None)
        t[f"fp8cast_{dn}_x"] = (x * 100).contiguous()
        t[f"fp8cast_{dn}_y"] = tq.fp8_eager(x * 100, None).contiguous()
        # reduce_amax
        xr = edges((6, 40, 24), dt, seed=4, scale=2.0)
        t[f"amax_{dn}_x"] = xr.contiguous()
        for name, ax in [("all", None), ("a0", [0]), ("a2", [2]), ("a01", [0, 1]), ("a02", [0, 2]), ("a12", [1, 2])]:
            t[f"amax_{dn}_{name}"] = reduce_amax(xr, axis=ax).contiguous()
    # special values, fp32
    sv = torch.tensor([448.0, 449.0, 463.99, 464.0, 465.0, 480.0, 1e9, 0.0, -0.0, 2.0**-9, 2.0**-10,
                       1.5 * 2.0**-10, 3.0, -5.5, 1e-20, 6e4])
    for a in [448.0, 3.0, 0.0, 1e-30]:
        t[f"fp8sv_{a}_y"] = tq.fp8_eager(sv, torch.tensor(a))
    t["fp8sv_x"] = sv
    save_file({k: v.contiguous() for k, v in t.items()}, str(OUT / "tensor_quant.safetensors"))
    (OUT / "tensor_quant.json").write_text(json.dumps(meta, indent=0))


def gen_quantizer():
    t = {}
    torch.manual_seed(10)

    def calib_then_quant(name, cfg, x, y=None):
        q = TensorQuantizer(QuantizerAttributeConfig(**cfg))
        q.enable_calib()
        q.disable_quant()
        q(x)
        q.load_calib_amax()
        q.disable_calib()
        q.enable_quant()
        out = q(x if y is None else y)
        t[name + "_x"] = x.contiguous()
        if y is not None:
            t[name + "_y_in"] = y.contiguous()
        t[name + "_amax"] = q.amax.contiguous()
        t[name + "_out"] = out.contiguous()

    for dn, dt in DT.items():
        x = edges((48, 256), dt, seed=11)
        y = edges((48, 256), dt, seed=12, scale=1.3)
        calib_then_quant(f"q_{dn}_int8_tensor", {"num_bits": 8}, x, y)
        calib_then_quant(f"q_{dn}_int8_axis0", {"num_bits": 8, "axis": 0}, x, y)
        calib_then_quant(f"q_{dn}_int8_axism1", {"num_bits": 8, "axis": -1}, x, y)
        calib_then_quant(f"q_{dn}_fp8_tensor", {"num_bits": (4, 3)}, x, y)
        calib_then_quant(f"q_{dn}_int4_b128", {"num_bits": 4, "block_sizes": {-1: 128, "type": "static"}}, x)
        calib_then_quant(f"q_{dn}_fp8_b128", {"num_bits": (4, 3), "block_sizes": {-1: 128}}, x)
    # padding / multi-axis block cases (tensor_quantizer_common.py:480-583)
    g = torch.Generator().manual_seed(13)
    a = torch.randn(3, 4, 5, generator=g)
    calib_then_quant("blk_simple_padding", {"num_bits": 8, "block_sizes": {-1: 2}}, a)
    b = torch.randn(2, 6, 4, generator=g)
    q = TensorQuantizer(QuantizerAttributeConfig(num_bits=8, block_sizes={-1: 2, 1: 3}))
    t["blk_complex_x"], t["blk_complex_out"] = b, q(b)
    c = torch.randn(2, 10, 5, generator=g)
    calib_then_quant("blk_complex_padding", {"num_bits": 8, "block_sizes": {-1: 2, 1: 3}}, c)
    # dynamic per-token FP8 (block_sizes {-1: None, type: dynamic})
    d = torch.randn(4, 7, 64, generator=g)
    q = TensorQuantizer(QuantizerAttributeConfig(num_bits=(4, 3), type="dynamic", block_sizes={-1: None, "type": "dynamic"}))
    t["fp8_per_token_x"], t["fp8_per_token_out"] = d, q(d)
    save_file(t, str(OUT / "quantizer.safetensors"))


def gen_calib():
    t, meta = {}, {}
    g = torch.Generator().manual_seed(20)
    xs = [torch.randn(32, 64, generator=g) * s for s in (1.0, 2.5, 0.7)]
    for i, x in enumerate(xs):
        t[f"batch{i}"] = x
    for name, axis in [("none", None), ("a0", 0), ("a1", 1)]:
        c = MaxCalibrator(8, axis, False)
        for x in xs:
            c.collect(x)
        t[f"max_{name}"] = c.compute_amax().contiguous()
    # histogram: growth on the second batch
    h = HistogramCalibrator(8, None, False, num_bins=256)
    for x in xs:
        h.collect(x)
    t["hist"] = h._calib_hist.clone()
    t["hist_edges"] = h._calib_bin_edges.clone()
    meta["hist_num_bins"] = h._num_bins
    meta["entropy"] = float(h.compute_amax("entropy", start_bin=128))
    meta["percentile_99"] = float(h.compute_amax("percentile", percentile=99.0))
    meta["percentile_9999"] = float(h.compute_amax("percentile", percentile=99.99))
    h2 = HistogramCalibrator(8, None, False, num_bins=2048, skip_zeros=True)
    xz = xs[0].clone()
    xz[:4] = 0
    h2.collect(xz)
    t["hist_skip_zeros"] = h2._calib_hist.clone()
    t["hist_skip_zeros_x"] = xz
    save_file(t, str(OUT / "calib.safetensors"))
    (OUT / "calib.json").write_text(json.dumps(meta, indent=1))


def gen_calib_ref():
    """HistogramCalibrator at its real semantics (calib/histogram.py:77-130, 285-325):
    * torch.histc's fp32 counts on 40 M-element peaked tensors (one bin > 2^24 per call), with 1
      and 3 intra-op threads (the per-thread fp32 saturation and the thread-order fold), a second
      call that grows the bins, and a skip_zeros case;
    * entropy / percentile / MSE amax from those histograms;
    * MSE amax for int 8 signed / unsigned and int 4 on the small ``calib`` batches -- the
      reference's ``fake_tensor_quant(centers, amax, num_bits, unsigned)`` call as it runs -- and
      the TypeError of the (4, 3) branch."""
    sys.path.insert(0, str(OUT))
    from hist_inputs import peaked

    t, meta = {}, {"cases": []}
    nthreads = torch.get_num_threads()
    for threads, skip in [(1, False), (3, False), (3, True)]:
        torch.set_num_threads(threads)
        h = HistogramCalibrator(8, None, False, num_bins=2048, skip_zeros=skip)
        for scale in (1.0, 1.5):
            h.collect(peaked(scale=scale, zeros_every=4 if skip else 0))
        key = f"t{threads}_skip{int(skip)}"
        t[f"hist_{key}"] = h._calib_hist.clone()
        t[f"edges_{key}"] = h._calib_bin_edges.clone()
        case = {"key": key, "threads": threads, "skip_zeros": skip, "num_bins": h._num_bins,
                "max_count": float(h._calib_hist.max())}
        case["percentile_9999"] = float(h.compute_amax("percentile", percentile=99.99))
        case["mse"] = float(h.compute_amax("mse"))
        if threads == 3 and not skip:
            case["entropy"] = float(h.compute_amax("entropy"))
        meta["cases"].append(case)
    torch.set_num_threads(nthreads)
    # MSE method on the small calib batches (int 8 / unsigned / int 4), FP8 raises
    g = torch.Generator().manual_seed(20)
    xs = [torch.randn(32, 64, generator=g) * s for s in (1.0, 2.5, 0.7)]
    for nb, u in [(8, False), (8, True), (4, False)]:
        h = HistogramCalibrator(nb, None, u, num_bins=256)
        for x in xs:
            h.collect(x.abs() if u else x)
        meta[f"small_mse_b{nb}_u{int(u)}"] = float(h.compute_amax("mse", start_bin=16))
    h = HistogramCalibrator((4, 3), None, False, num_bins=256)
    h.collect(xs[0])
    try:
        h.compute_amax("mse", start_bin=16)
        meta["fp8_mse_error"] = None
    except TypeError as e:
        meta["fp8_mse_error"] = "TypeError: " + str(e)
    save_file(t, str(OUT / "calib_ref.safetensors"))
    (OUT / "calib_ref.json").write_text(json.dumps(meta, indent=1))


def gen_mtq_linear():
    torch.manual_seed(30)
    m = nn.Linear(1024, 1024)
    w0 = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(31)
    calib = [torch.randn(16, 1024, generator=g) for _ in range(4)]
    test = torch.randn(8, 1024, generator=g)

    def loop(model):
        for c in calib:
            model(c)

    mtq.quantize(m, mtq.INT8_DEFAULT_CFG, loop)
    t = {"weight": w0["weight"], "bias": w0["bias"], "test": test, "out": m(test).detach()}
    for i, c in enumerate(calib):
        t[f"calib{i}"] = c
    t["input_amax"] = m.input_quantizer.amax.clone()
    t["weight_amax"] = m.weight_quantizer.amax.clone()
    save_file(t, str(OUT / "mtq_linear.safetensors"))


def tiny_llama():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(
        hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=4,
        num_key_value_heads=2, vocab_size=32, max_position_embeddings=64,
    )
    torch.manual_seed(40)
    return LlamaForCausalLM(cfg).eval()


def gen_llama_fp8():
    model = tiny_llama()
    sd = {k: v.clone().contiguous() for k, v in model.state_dict().items()}
    g = torch.Generator().manual_seed(41)
    ids = torch.randint(0, 32, (4, 2, 16), generator=g)
    test = torch.randint(0, 32, (2, 16), generator=g)

    def loop(mm):
        for b in ids:
            mm(b)

    mtq.quantize(model, mtq.FP8_DEFAULT_CFG, loop)
    t = {f"sd.{k}": v for k, v in sd.items()}
    t["calib_ids"] = ids
    t["test_ids"] = test
    t["logits"] = model(test).logits.detach()
    for n, q in model.named_modules():
        if isinstance(q, TensorQuantizer) and q.amax is not None:
            t[f"amax.{n}"] = q.amax.clone().contiguous()
    save_file(t, str(OUT / "llama_fp8.safetensors"))


def tiny_mixtral():
    from transformers import MixtralConfig, MixtralForCausalLM

    cfg = MixtralConfig(
        hidden_size=32, intermediate_size=48, num_hidden_layers=2, num_attention_heads=4,
        num_key_value_heads=2, vocab_size=32, max_position_embeddings=64, num_local_experts=4,
        num_experts_per_tok=2,
    )
    torch.manual_seed(60)
    return MixtralForCausalLM(cfg).eval()


def gen_mixtral_fp8():
    """Fused-experts MoE path (plugins/huggingface.py _QuantFusedExperts) under FP8_DEFAULT_CFG."""
    model = tiny_mixtral()
    sd = {k: v.clone().contiguous() for k, v in model.state_dict().items()}
    g = torch.Generator().manual_seed(61)
    ids = torch.randint(0, 32, (4, 2, 16), generator=g)
    test = torch.randint(0, 32, (2, 16), generator=g)

    def loop(mm):
        for b in ids:
            mm(b)

    mtq.quantize(model, mtq.FP8_DEFAULT_CFG, loop)
    t = {f"sd.{k}": v for k, v in sd.items()}
    t["calib_ids"] = ids
    t["test_ids"] = test
    t["logits"] = model(test).logits.detach()
    names = []
    for n, q in model.named_modules():
        if isinstance(q, TensorQuantizer):
            names.append([n, bool(q.is_enabled)])
            if q.amax is not None:
                t[f"amax.{n}"] = q.amax.clone().contiguous()
    save_file(t, str(OUT / "mixtral_fp8.safetensors"))
    (OUT / "mixtral_fp8.json").write_text(json.dumps({"quantizers": names}, indent=0))


sys.path.insert(0, str(OUT))
from prod_models import PROD_CASES, fingerprint as _fingerprint, prod_inputs, prod_model, sha as _sha  # noqa: E402


def _prod_case(kind, seed, cfg_name, algorithm=None):
    import copy

    model = prod_model(kind, seed)
    fp = _fingerprint(model)
    ids, test = prod_inputs(seed)
    cfg = copy.deepcopy(getattr(mtq, cfg_name))
    if algorithm is not None:
        cfg["algorithm"] = algorithm

    def loop(mm):
        for b in ids:
            mm(b)

    with torch.no_grad():
        mtq.quantize(model, cfg, loop)
        logits = model(test).logits.float()
    t = {"calib_ids": ids, "test_ids": test, "logits": logits}
    meta = {"kind": kind, "seed": seed, "config": cfg_name, "algorithm": algorithm, "fingerprint": fp,
            "threads": torch.get_num_threads(), "amax_sha": {}, "weight_sha": {}, "awq": {}}
    for n, q in model.named_modules():
        if isinstance(q, TensorQuantizer) and q.is_enabled and q.amax is not None:
            a = q.amax.detach()
            if a.numel() <= 65536:
                t[f"amax.{n}"] = a.clone().contiguous()
            else:  # static block amax (INT4 block 128: 1.8 M values per layer): bytes pinned by hash
                meta["amax_sha"][n] = [_sha(a), str(a.dtype), list(a.shape)]
    for n, m in model.named_modules():
        if hasattr(m, "awq_lite"):
            h = m.awq_lite
            meta["awq"][n] = {"best_alpha": h.best_alpha, "N": m.weight.shape[0], "K": m.weight.shape[1]}
            t[f"act_scale.{n}"] = h.act_scale.clone()
            t[f"best_scale.{n}"] = h.best_scale.clone()
            meta["weight_sha"][n] = _sha(m.weight)
    return t, meta


def gen_prod():
    """End-to-end parity at production dispatch sizes: mtq.quantize on a
    2-layer Llama with Llama-3-8B layer shapes (hidden 4096, intermediate 14336, 32 / 8 heads) under
    FP8_DEFAULT_CFG (per-tensor), INT8_DEFAULT_CFG (per-channel weights) and INT4_AWQ_CFG (awq_lite,
    block 128), and a 1-layer Mixtral (hidden 1024, 8 experts) under FP8_DEFAULT_CFG, in bf16.
    Weights are regenerated from the seed (their sha256 is stored), so only inputs, amax, AWQ
    scales and logits are kept."""
    tensors, meta = {}, {}
    for name, (kind, seed, cfg_name, algo) in PROD_CASES.items():
        print("  prod case", name, flush=True)
        t, m = _prod_case(kind, seed, cfg_name, algo)
        tensors.update({f"{name}.{k}": v for k, v in t.items()})
        meta[name] = m
    save_file(tensors, str(OUT / "prod.safetensors"))
    (OUT / "prod.json").write_text(json.dumps(meta, indent=0))


class _SimpleMLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 16), nn.ReLU(), nn.Linear(16, 16))

    def forward(self, x):
        return self.net(x)


def gen_awq():
    torch.manual_seed(50)
    model = _SimpleMLP()
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    g = torch.Generator().manual_seed(51)
    data = [torch.randn(2, 16, generator=g) for _ in range(4)]
    cfg = {
        "quant_cfg": [
            {"quantizer_name": "*", "enable": False},
            {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4, "block_sizes": {-1: 8, "type": "static"}}},
        ],
        "algorithm": {"method": "awq_lite", "alpha_step": 0.1, "debug": True},
    }

    def loop(mm):
        for d in data:
            mm(d)

    mtq.quantize(model, cfg, loop)
    t = {f"sd.{k}": v for k, v in sd.items()}
    for i, d in enumerate(data):
        t[f"data{i}"] = d
    meta = {}
    for n, m in model.named_modules():
        if hasattr(m, "awq_lite"):
            t[f"best_scale.{n}"] = m.awq_lite.best_scale.clone()
            t[f"weight.{n}"] = m.weight.detach().clone()
            t[f"wamax.{n}"] = m.weight_quantizer.amax.clone()
            t[f"pqs.{n}"] = m.input_quantizer.pre_quant_scale.clone()
            meta[n] = {"best_alpha": m.awq_lite.best_alpha, "loss": {str(k): float(v) for k, v in m.awq_lite.loss.items()}}
    test = torch.randn(3, 16, generator=g)
    t["test"] = test
    t["out"] = model(test).detach()
    save_file(t, str(OUT / "awq.safetensors"))
    (OUT / "awq.json").write_text(json.dumps(meta, indent=1))


class _WideMLP(nn.Module):
    """K % 128 == 0 everywhere; output widths on both sides of the fused-search crossover
    (N = 2304 above it; 256 and 1024 at or below it), one linear without bias."""

    def __init__(self):
        super().__init__()
        self.net = nn.Sequential(
            nn.Linear(256, 2304), nn.ReLU(), nn.Linear(2304, 256), nn.ReLU(),
            nn.Linear(256, 1024, bias=False), nn.ReLU(), nn.Linear(1024, 256),
        )

    def forward(self, x):
        return self.net(x)


def awq_b128_inputs():
    """bf16 MLP + calibration batches of the INT4_AWQ_CFG (block 128) golden: channels of the input
    carry per-column gains (0.25 .. 8) so act_scale varies across K, M = 192 rows per batch (a
    tail below the 256-row tile)."""
    torch.manual_seed(73)
    model = _WideMLP().to(torch.bfloat16)
    g = torch.Generator().manual_seed(71)
    gain = torch.exp2(torch.rand(256, generator=g) * 5 - 2)
    data = [(torch.randn(2, 96, 256, generator=g) * gain).to(torch.bfloat16) for _ in range(3)]
    test = (torch.randn(2, 32, 256, generator=g) * gain).to(torch.bfloat16)
    return model, data, test


def gen_awq_b128():
    """C3's real search path: mtq.INT4_AWQ_CFG (awq_lite, block 128, alpha step 0.1) in bf16 on
    linears that qualify for the fast search (K % 64 == 0) -- the product's fused-MFMA and
    batched paths are pinned against this run of the reference."""
    model, data, test = awq_b128_inputs()
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    import copy

    cfg = copy.deepcopy(mtq.INT4_AWQ_CFG)
    cfg["algorithm"] = {"method": "awq_lite", "alpha_step": 0.1, "debug": True}

    def loop(mm):
        for d in data:
            mm(d)

    mtq.quantize(model, cfg, loop)
    t = {f"sd.{k}": v for k, v in sd.items()}
    for i, d in enumerate(data):
        t[f"data{i}"] = d
    meta = {"cfg_algorithm": cfg["algorithm"], "threads": torch.get_num_threads()}
    for n, m in model.named_modules():
        if hasattr(m, "awq_lite"):
            t[f"best_scale.{n}"] = m.awq_lite.best_scale.clone()
            t[f"act_scale.{n}"] = m.awq_lite.act_scale.clone()
            t[f"weight_scale.{n}"] = m.awq_lite.weight_scale.clone()
            t[f"weight.{n}"] = m.weight.detach().clone()
            t[f"wamax.{n}"] = m.weight_quantizer.amax.clone()
            t[f"pqs.{n}"] = m.input_quantizer.pre_quant_scale.clone()
            meta[n] = {"best_alpha": m.awq_lite.best_alpha,
                       "loss": {str(k): float(v) for k, v in m.awq_lite.loss.items()},
                       "N": m.weight.shape[0], "K": m.weight.shape[1]}
    t["test"] = test
    t["out"] = model(test).detach()
    save_file(t, str(OUT / "awq_b128.safetensors"))
    (OUT / "awq_b128.json").write_text(json.dumps(meta, indent=1))


def gen_nvfp4():
    """NVFP4 dynamic two-level fake quant from the reference's own Triton kernel
    (kernels/quantization/gemm/fp4_kernel_hopper.py fp4_fake_quant_block), run on CPU with the
    Triton interpreter (TRITON_INTERPRET=1; its cuda-device context is bypassed for CPU tensors).

    The Triton 3.6 interpreter's casts are not all the hardware's.  Its fp32 -> bf16 store
    truncates (handled by running the kernel in fp32 and rounding with torch, see below).  Its
    fp32 -> float8e4nv cast it truncates where
    round-to-nearest carries into the next binade (1.97 -> 1.0, not 2.0) and flushes small values
    to 0 (checked below against torch's RNE cast, which is what cvt.rn.satfinite computes).  The
    per-block scale goes through that cast, so the blocks whose scale hits such a value are
    recorded in ``mask`` and excluded from the comparison; everything else is pinned."""
    import contextlib
    import importlib

    import triton
    import triton.language as tl

    torch.cuda.device = lambda d: contextlib.nullcontext()  # the wrapper's context, CPU tensors
    hop = importlib.import_module("modelopt.torch.kernels.quantization.gemm.fp4_kernel_hopper")

    @triton.jit
    def _cast_fp8(x_ptr, y_ptr, n, BLOCK: tl.constexpr):
        o = tl.arange(0, BLOCK)
        x = tl.load(x_ptr + o, mask=o < n, other=0.0)
        tl.store(y_ptr + o, x.to(tl.float8e4nv).to(tl.float32), mask=o < n)

    def interp_cast_ok(s8):
        flat = s8.reshape(-1).contiguous()
        out = torch.empty_like(flat)
        blk = triton.next_power_of_2(max(flat.numel(), 1))
        _cast_fp8[(1,)](flat, out, flat.numel(), BLOCK=blk)
        return (out == flat.to(torch.float8_e4m3fn).float()).reshape(s8.shape)

    t, meta = {}, {}
    g = torch.Generator().manual_seed(70)
    cases = [("f32_64x64", torch.float32, (64, 64)), ("bf16_48x96", torch.bfloat16, (48, 96)),
             ("f16_32x80", torch.float16, (32, 80)), ("bf16_16x40", torch.bfloat16, (16, 40)),
             ("f32_8x16_zero", torch.float32, (8, 16))]
    for name, dt, shape in cases:
        x = (torch.randn(shape, generator=g) * torch.logspace(-2, 1, shape[-1])).to(dt)
        if name.endswith("zero"):
            x[0] = 0
            x[1, :4] = -0.0
        ga = x.float().abs().amax()
        # the kernel loads x and computes in fp32; its final fp32 -> bf16 store in the interpreter
        # truncates instead of rounding to nearest like the hardware cast, so the fp32 result is
        # taken and rounded with torch's RNE cast (exact for x itself: bf16/f16 -> fp32 is exact)
        y = hop.fp4_fake_quant_block(x.float(), ga).to(dt)
        # which blocks' scales the interpreter casts correctly
        xf = x.float()
        pad = (-shape[-1]) % 16
        xp = torch.nn.functional.pad(xf, (0, pad)) if pad else xf
        bmax = xp.reshape(shape[0], -1, 16).abs().amax(-1)
        gs = ga / torch.tensor(2688.0)
        gs = torch.where(gs > 0, gs, torch.tensor(1e-12))
        s8 = torch.minimum(bmax / (torch.tensor(6.0) * gs), torch.tensor(448.0))
        ok = interp_cast_ok(s8)
        t[f"{name}.x"], t[f"{name}.amax"], t[f"{name}.y"] = x, ga.reshape(1), y
        t[f"{name}.block_ok"] = ok.to(torch.uint8)
        meta[name] = {"blocks": int(ok.numel()), "excluded": int((~ok).sum())}
    # static two-level path (fp4_kernel.py static_blockwise_fp4_fake_quant): its element kernel
    # calls libdevice.isnan, which the Triton interpreter cannot run, so the golden pins the
    # reference's scale computation (compute_fp4_scales: amax/6, FP8-quantised through the
    # reference's scaled_e4m3_impl) -- the element pass is the same fp4_round_magnitude the
    # dynamic golden above pins
    fk = importlib.import_module("modelopt.torch.kernels.quantization.gemm.fp4_kernel")
    for name, shape in [("static_scales_a", (64, 1)), ("static_scales_b", (300, 1))]:
        amax = (torch.rand(shape, generator=g) * torch.logspace(-4, 1, shape[0]).view(-1, 1)).float()
        amax[0] = 0.0
        t[f"{name}.amax"] = amax
        t[f"{name}.scale"] = fk.compute_fp4_scales(amax, amax.amax(), True, 448.0)
        t[f"{name}.scale_g2"] = fk.compute_fp4_scales(amax, amax.amax() * 2, True, 448.0)
        t[f"{name}.scale_46"] = fk.compute_fp4_scales(amax, None, True, 256.0)
        meta[name] = {"static_scales": True}
    save_file(t, str(OUT / "nvfp4.safetensors"))
    (OUT / "nvfp4.json").write_text(json.dumps(meta, indent=1))


def tiny_llama_export():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(
        hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
        num_key_value_heads=2, vocab_size=32, max_position_embeddings=64,
        architectures=["LlamaForCausalLM"],
    )
    torch.manual_seed(80)
    return LlamaForCausalLM(cfg).eval()


EXPORT_CASES = {
    "fp8": "FP8_DEFAULT_CFG",
    "fp8_pcpt": "FP8_PER_CHANNEL_PER_TOKEN_CFG",
    "int8_sq": "INT8_DEFAULT_CFG",
    "int4_awq": "INT4_AWQ_CFG",
    "w4a8_awq": "W4A8_AWQ_BETA_CFG",
    "nvfp4": "NVFP4_DEFAULT_CFG",
    "mxfp4": "MXFP4_DEFAULT_CFG",
    "mxfp8": "MXFP8_DEFAULT_CFG",
    "fp8_pb_wo": "FP8_2D_BLOCKWISE_WEIGHT_ONLY_CFG",
    "int8_wo": "INT8_WEIGHT_ONLY_CFG",
    "w4a16_nvfp4": "W4A16_NVFP4_CFG",
    "w4a8_nvfp4_fp8": "W4A8_NVFP4_FP8_CFG",
    "w4a8_mxfp4_fp8": "W4A8_MXFP4_FP8_CFG",
}


def export_cfg(name):
    """The preset, with INT4 groups of 32 so the tiny model (hidden 64) has two per row, and FP8 2D
    blocks of 32 x 32 (the preset's 128 x 128 would pad every weight of the tiny model)."""
    import copy

    cfg = copy.deepcopy(getattr(mtq, EXPORT_CASES[name]))
    for e in cfg["quant_cfg"]:
        if e.get("quantizer_name") == "*weight_quantizer":
            c = e["cfg"]
            first = c[0] if isinstance(c, list) else c
            if first.get("num_bits") == 4:
                first["block_sizes"] = {-1: 32, "type": "static"}
            if first.get("num_bits") == (4, 3) and -2 in (first.get("block_sizes") or {}):
                first["block_sizes"] = {-1: 32, -2: 32}
    return cfg


def tiny_mixtral_export():
    from transformers import MixtralConfig, MixtralForCausalLM

    cfg = MixtralConfig(
        hidden_size=64, intermediate_size=64, num_hidden_layers=2, num_attention_heads=4,
        num_key_value_heads=2, vocab_size=32, max_position_embeddings=64, num_local_experts=4,
        num_experts_per_tok=2, architectures=["MixtralForCausalLM"],
    )
    torch.manual_seed(82)
    return MixtralForCausalLM(cfg).eval()


EXPORT_MOE_CASES = {"moe_fp8": "FP8_DEFAULT_CFG", "moe_nvfp4": "NVFP4_DEFAULT_CFG"}


def gen_export():
    """Unified HF checkpoint export (export/unified_export_hf.py export_hf_checkpoint) of a tiny
    Llama per format: the post-calibration state (weights + quantizer buffers) and the exported
    files (model.safetensors tensors, hf_quant_config.json, config.json quantization_config)."""
    import tempfile

    from safetensors.torch import load_file

    from modelopt.torch.export import export_hf_checkpoint

    g = torch.Generator().manual_seed(81)
    ids = torch.randint(0, 32, (4, 2, 16), generator=g)
    t, meta = {"calib_ids": ids}, {}
    for name in list(EXPORT_CASES) + list(EXPORT_MOE_CASES):
        moe = name in EXPORT_MOE_CASES
        m = tiny_mixtral_export() if moe else tiny_llama_export()
        cfg = getattr(mtq, EXPORT_MOE_CASES[name]) if moe else export_cfg(name)
        mtq.quantize(m, cfg, lambda mm: [mm(b) for b in ids])
        for k, v in m.state_dict().items():
            t[f"{name}.state.{k}"] = v.detach().clone().contiguous()
        with tempfile.TemporaryDirectory() as d:
            export_hf_checkpoint(m, export_dir=d)
            for k, v in load_file(os.path.join(d, "model.safetensors")).items():
                t[f"{name}.export.{k}"] = v.contiguous()
            hq = json.load(open(os.path.join(d, "hf_quant_config.json")))
            cq = json.load(open(os.path.join(d, "config.json"))).get("quantization_config")
        hq["producer"]["version"] = None
        if cq and "producer" in cq:
            cq["producer"]["version"] = None
        meta[name] = {"preset": (EXPORT_MOE_CASES if moe else EXPORT_CASES)[name], "model": "mixtral" if moe else "llama",
                      "hf_quant_config": hq, "quantization_config": cq}
    save_file(t, str(OUT / "export.safetensors"))
    (OUT / "export.json").write_text(json.dumps(meta, indent=1))


def gen_mse():
    """MSE weight calibration (calib/mse.py, model_calib.py:733-827).

    * ``sweep.*``: the reference's fused NVFP4 FP8-scale sweep Triton kernel
      (kernels/quantization/gemm/nvfp4_fp8_sweep.py ``_fp8_scale_sweep_kernel``) run on CPU via the
      Triton interpreter (fp32 arithmetic only -- none of the interpreter's cast quirks apply), on
      ``[n_blocks, block]`` weights (the wrapper's CUDA check is bypassed by calling the kernel).
    * ``cal.*``: ``MseCalibrator`` multiplier search with the reference TensorQuantizer as
      quant_func (per-tensor FP8, per-channel INT8, static-block INT4), incl. every candidate's loss.
    * ``model.*``: ``mtq.quantize(tiny Llama, {"method": "mse"})`` weight amaxes for INT8 / FP8.
    """
    import copy
    from functools import partial

    import triton

    from modelopt.torch.kernels.quantization.gemm import _fp8_scale_candidates as cand_mod
    from modelopt.torch.kernels.quantization.gemm import nvfp4_fp8_sweep as sweep_mod
    from modelopt.torch.quantization.calib import MseCalibrator
    from modelopt.torch.quantization.model_calib import _mse_quant_func

    t, meta = {}, {"sweep": {}, "cal": {}, "model": {}}
    g = torch.Generator().manual_seed(90)
    kern = sweep_mod._fp8_scale_sweep_kernel.fn  # the JIT function under the autotuner
    cases = [("f32_b16", torch.float32, 512, 16), ("bf16_b16", torch.bfloat16, 640, 16),
             ("f16_b16", torch.float16, 256, 16), ("f32_b32", torch.float32, 128, 32),
             ("bf16_b8", torch.bfloat16, 256, 8), ("f32_zero", torch.float32, 16, 16)]
    for name, dt, nb, bs in cases:
        x = (torch.randn(nb, bs, generator=g) * torch.logspace(-3, 1, nb)[:, None]).to(dt)
        if name == "f32_zero":
            x.zero_()
        elif name.startswith("bf16_b16"):
            x[3] = 0
            x[5, :] = x[5, 0]  # all-equal magnitudes
        ga = x.float().abs().amax()
        cands = cand_mod.fp8_scale_candidates("cpu").float()
        best = torch.empty(nb, dtype=torch.float32)
        kern[(triton.cdiv(nb, 16),)](x.contiguous().view(-1), cands, ga.reshape(1), best, nb,
                                     BLOCK_SIZE=bs, NUM_CANDIDATES=int(cands.numel()),
                                     BLOCKS_PER_PROGRAM=16)
        t[f"sweep.{name}.x"], t[f"sweep.{name}.global_amax"], t[f"sweep.{name}.best"] = x, ga.reshape(()), best
        meta["sweep"][name] = {"blocks": nb, "block": bs}
    t["sweep.candidates"] = cand_mod.fp8_scale_candidates("cpu").float()

    # MseCalibrator with the reference quantizer as quant_func
    qcases = [("fp8_tensor", {"num_bits": (4, 3), "axis": None}, torch.float32, (64, 128)),
              ("int8_ch", {"num_bits": 8, "axis": 0}, torch.float32, (48, 96)),
              ("int8_ch_bf16", {"num_bits": 8, "axis": 0}, torch.bfloat16, (32, 128)),
              ("int4_blk", {"num_bits": 4, "block_sizes": {-1: 32, "type": "static"}}, torch.float32, (16, 128)),
              ("fp8_tensor_bf16", {"num_bits": (4, 3), "axis": None}, torch.bfloat16, (64, 64))]
    for name, qc, dt, shape in qcases:
        w = (torch.randn(shape, generator=g) * torch.logspace(-1, 0.5, shape[0])[:, None]).to(dt)
        w[0, 0] = 8.0  # an outlier for the clipping trade-off
        q = TensorQuantizer(QuantizerAttributeConfig(**qc))
        q.enable_calib(); q.disable_quant()
        q(w)
        q.load_calib_amax()
        q.disable_calib(); q.enable_quant()
        init = q._amax.clone()
        cal = MseCalibrator(amax=init, axis=q._calibrator._axis, quant_func=partial(_mse_quant_func, quantizer=q))
        q._calibrator = cal
        q.enable_calib(); q.disable_quant()
        q(w)
        losses = torch.stack([ls.reshape(-1) for ls in cal._losses_sum])
        best = cal.compute_amax()
        t[f"cal.{name}.w"], t[f"cal.{name}.init_amax"] = w, init
        t[f"cal.{name}.losses"], t[f"cal.{name}.best"] = losses, best.clone()
        t[f"cal.{name}.candidates"] = cal._candidates.clone()
        meta["cal"][name] = {"cfg": {k: (list(v) if isinstance(v, tuple) else v) for k, v in qc.items() if k != "block_sizes"},
                             "block": (qc.get("block_sizes") or {}).get(-1), "dtype": str(dt), "axis": q._calibrator._axis}

    # end to end: mtq.quantize with {"method": "mse"}
    g2 = torch.Generator().manual_seed(91)
    ids = torch.randint(0, 32, (2, 2, 16), generator=g2)
    t["model.calib_ids"] = ids
    for name, preset in [("int8", "INT8_DEFAULT_CFG"), ("fp8", "FP8_DEFAULT_CFG")]:
        m = tiny_llama()
        cfg = copy.deepcopy(getattr(mtq, preset))
        cfg["algorithm"] = {"method": "mse"}
        mtq.quantize(m, cfg, lambda mm: [mm(b) for b in ids])
        for n, mod in m.named_modules():
            if isinstance(mod, TensorQuantizer) and mod.is_enabled and getattr(mod, "_amax", None) is not None:
                t[f"model.{name}.{n}"] = mod._amax.clone()
        meta["model"][name] = preset
    save_file(t, str(OUT / "mse.safetensors"))
    (OUT / "mse.json").write_text(json.dumps(meta, indent=1))


class _ClipMLP(nn.Module):
    """The reference AWQ tests' toy model shape (test_calib.py:38-56): bias-free 16 -> f1 -> f2 -> 16."""

    def __init__(self, f1=32, f2=16):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(16, f1, bias=False), nn.ReLU(), nn.Linear(f1, f2, bias=False),
                                 nn.ReLU(), nn.Linear(f2, 16, bias=False))

    def forward(self, x):
        return self.net(x)


def gen_awq_clip():
    """AWQ-clip / AWQ-full (model_calib.py:1725-1940) on the reference test's _SimpleMLP (INT4,
    block 8; test_calib.py:125-283), a padded variant (ci not a multiple of the block) and a bf16
    linear with block 128 (the products and sums rounded to bf16 as the reference's
    ``(inputs * w).sum(-1)``), with debug=True so every per-shrink loss is recorded."""
    import copy

    def awq_cfg(method, block):
        cfg = copy.deepcopy(mtq.INT4_AWQ_CFG)
        for e in cfg["quant_cfg"]:
            if e.get("quantizer_name") == "*weight_quantizer":
                e["cfg"]["block_sizes"] = {-1: block, "type": "static"}
        cfg["algorithm"] = {"method": method, "debug": True}
        if method != "awq_clip":
            cfg["algorithm"]["alpha_step"] = 0.1
        return cfg

    t, meta = {}, {}
    g = torch.Generator().manual_seed(95)

    def record(name, model, data, test):
        t[f"{name}.test"] = test
        for n, mod in model.named_modules():
            if hasattr(mod, "awq_clip"):
                h = mod.awq_clip
                t[f"{name}.{n}.w_amax"] = h.w_amax.clone()
                t[f"{name}.{n}.best_clip"] = h.best_clip_val.clone()
                t[f"{name}.{n}.losses"] = torch.stack([v.reshape(-1) for v in h.loss.values()])
                t[f"{name}.{n}.amax"] = mod.weight_quantizer.amax.clone()
                t[f"{name}.{n}.weight"] = mod.weight.detach().clone()
                if mod.input_quantizer.pre_quant_scale is not None:
                    t[f"{name}.{n}.pqs"] = mod.input_quantizer.pre_quant_scale.clone()
                meta[name]["layers"][n] = {"shrinks": [float(k) for k in h.loss], "num_tokens": int(h.num_tokens)}
        with torch.no_grad():
            t[f"{name}.out"] = model(test.clone()).detach()

    for name, method, f1, f2, block in [("mlp_clip", "awq_clip", 32, 16, 8), ("mlp_full", "awq_full", 32, 16, 8),
                                        ("mlp_full_pad", "awq_full", 13, 19, 8)]:
        torch.manual_seed(96)
        model = _ClipMLP(f1=f1, f2=f2)
        t[f"{name}.sd"] = torch.cat([v.reshape(-1) for v in model.state_dict().values()])
        for k, v in model.state_dict().items():
            t[f"{name}.sd.{k}"] = v.clone()
        data = [torch.randn(2, 64, 16, generator=g) for _ in range(2)]
        for i, d in enumerate(data):
            t[f"{name}.data{i}"] = d
        meta[name] = {"method": method, "block": block, "f1": f1, "f2": f2, "layers": {}}
        mtq.quantize(model, awq_cfg(method, block), lambda mm: [mm(d.clone()) for d in data])
        record(name, model, data, torch.randn(3, 16, generator=g))

    # bf16 linear, block 128, 3 batches of 4 x 80 tokens (stride-sampled to 64 per batch)
    name = "bf16_lin"
    torch.manual_seed(97)
    lin = nn.Sequential(nn.Linear(384, 192, bias=False)).to(torch.bfloat16)
    for k, v in lin.state_dict().items():
        t[f"{name}.sd.{k}"] = v.clone()
    data = [torch.randn(4, 80, 384, generator=g).to(torch.bfloat16) for _ in range(3)]
    for i, d in enumerate(data):
        t[f"{name}.data{i}"] = d
    meta[name] = {"method": "awq_clip", "block": 128, "layers": {}}
    mtq.quantize(lin, awq_cfg("awq_clip", 128), lambda mm: [mm(d) for d in data])
    record(name, lin, data, torch.randn(2, 384, generator=g).to(torch.bfloat16))
    save_file(t, str(OUT / "awq_clip.safetensors"))
    (OUT / "awq_clip.json").write_text(json.dumps(meta, indent=1))


def kv_cfg(name):
    """FP8 weights/activations plus the attention BMM quantizers of each KV case."""
    import copy

    cfg = copy.deepcopy(mtq.FP8_DEFAULT_CFG)
    fp8 = {"num_bits": (4, 3), "axis": None}
    extra = {
        "fp8_kv": [{"quantizer_name": "*[kv]_bmm_quantizer", "cfg": dict(fp8)}],
        "fp8_kv_cast": [{"quantizer_name": "*[kv]_bmm_quantizer", "cfg": dict(fp8, use_constant_amax=True)}],
        "qkv_fp8": [{"quantizer_name": "*[qkv]_bmm_quantizer", "cfg": dict(fp8)}],
        "int8_kv": [{"quantizer_name": "*[kv]_bmm_quantizer", "cfg": {"num_bits": 8, "axis": None}}],
    }[name]
    cfg["quant_cfg"] = cfg["quant_cfg"] + extra
    return cfg


def gen_kv():
    """KV-cache / attention BMM quantizers (plugins/huggingface.py:78-410 _QuantAttention): tiny
    Llama (sdpa attention) with FP8 W/A plus FP8 K/V (calibrated and constant-amax "cast"), FP8
    Q/K/V, INT8 K/V: every quantizer amax, logits, and the unified HF export (k_scale / v_scale,
    kv_cache_quant_algo)."""
    import tempfile

    from safetensors.torch import load_file

    from modelopt.torch.export import export_hf_checkpoint

    g = torch.Generator().manual_seed(85)
    ids = torch.randint(0, 32, (3, 2, 16), generator=g)
    test = torch.randint(0, 32, (2, 16), generator=g)
    t, meta = {"calib_ids": ids, "test_ids": test}, {}
    for name in ["fp8_kv", "fp8_kv_cast", "qkv_fp8", "int8_kv"]:
        m = tiny_llama_export()
        mtq.quantize(m, kv_cfg(name), lambda mm: [mm(b) for b in ids])
        for k, v in m.state_dict().items():
            t[f"{name}.state.{k}"] = v.detach().clone().contiguous()
        enabled = []
        for n, q in m.named_modules():
            if isinstance(q, TensorQuantizer) and q.is_enabled:
                enabled.append(n)
                if getattr(q, "_amax", None) is not None:
                    t[f"{name}.amax.{n}"] = q._amax.clone().contiguous()
        with torch.no_grad():
            t[f"{name}.logits"] = m(test).logits.detach()
        meta[name] = {"enabled": enabled}
        if name in ("fp8_kv", "fp8_kv_cast"):
            with tempfile.TemporaryDirectory() as d:
                export_hf_checkpoint(m, export_dir=d)
                for k, v in load_file(os.path.join(d, "model.safetensors")).items():
                    t[f"{name}.export.{k}"] = v.contiguous()
                hq = json.load(open(os.path.join(d, "hf_quant_config.json")))
                cq = json.load(open(os.path.join(d, "config.json"))).get("quantization_config")
            hq["producer"]["version"] = None
            if cq and "producer" in cq:
                cq["producer"]["version"] = None
            meta[name].update(hf_quant_config=hq, quantization_config=cq)
    save_file(t, str(OUT / "kv.safetensors"))
    (OUT / "kv.json").write_text(json.dumps(meta, indent=1))


def gen_presets():
    names = [
        "INT8_DEFAULT_CFG", "INT8_WEIGHT_ONLY_CFG", "FP8_DEFAULT_CFG", "FP8_PER_CHANNEL_PER_TOKEN_CFG",
        "FP8_2D_BLOCKWISE_WEIGHT_ONLY_CFG", "INT4_BLOCKWISE_WEIGHT_ONLY_CFG", "INT4_AWQ_CFG",
        "MXFP8_DEFAULT_CFG", "MXFP6_DEFAULT_CFG", "MXFP4_DEFAULT_CFG", "MXINT8_DEFAULT_CFG",
        "W4A8_MXFP4_FP8_CFG", "MXFP4_MLP_WEIGHT_ONLY_CFG", "NVFP4_DEFAULT_CFG", "NVFP4_AWQ_LITE_CFG",
        "W4A8_AWQ_BETA_CFG", "FP8_KV_CFG", "NVFP4_KV_CFG", "NVFP4_AWQ_CLIP_CFG", "NVFP4_AWQ_FULL_CFG",
        "NVFP4_W4A4_WEIGHT_MSE_FP8_SWEEP_CFG", "FP8_AFFINE_KV_CFG", "NVFP4_AFFINE_KV_CFG", "NVFP4_FP8_MHA_CONFIG",
        "W4A16_NVFP4_CFG", "W4A8_NVFP4_FP8_CFG", "NVFP4_MLP_ONLY_CFG", "NVFP4_OMLP_ONLY_CFG", "NVFP4_EXPERTS_ONLY_CFG",
        "NVFP4_MLP_WEIGHT_ONLY_CFG", "MAMBA_MOE_FP8_AGGRESSIVE_CFG", "MAMBA_MOE_FP8_CONSERVATIVE_CFG",
        "MAMBA_MOE_NVFP4_AGGRESSIVE_CFG", "MAMBA_MOE_NVFP4_CONSERVATIVE_CFG", "NVFP4_FOUR_OVER_SIX_CFG",
        "INT8_SMOOTHQUANT_CFG", "NVFP4_SVDQUANT_DEFAULT_CFG", "NVFP4_W4A4_WEIGHT_LOCAL_HESSIAN_CFG",
        "NVFP4_KV_ROTATE_CFG",
    ]

    def enc(o):
        if isinstance(o, dict):
            return {("__int__" + str(k)) if isinstance(k, int) else k: enc(v) for k, v in o.items()}
        if isinstance(o, (list, tuple)):
            return {"__tuple__": [enc(v) for v in o]} if isinstance(o, tuple) else [enc(v) for v in o]
        return o

    (OUT / "presets.json").write_text(json.dumps({n: enc(getattr(mtq, n)) for n in names}, indent=0))


def gen_mx_kat():
    """Extract the literal in/out tables of the reference MX known-answer tests (data only)."""
    src = (REF / "tests/gpu/torch/quantization/test_quantize_mxformats_cuda.py").read_text()
    tree = ast.parse(src)
    kats = {}
    for fn in tree.body:
        if not isinstance(fn, ast.FunctionDef) or fn.name not in ("test_mxfp4", "test_mxfp6", "test_mxfp8", "test_mxint8"):
            continue
        tables, calls = [], []
        for node in ast.walk(fn):
            if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "tensor" and node.args:
                try:
                    tables.append((node.lineno, ast.literal_eval(node.args[0])))
                except ValueError:
                    pass
            if isinstance(node, ast.Subscript) and getattr(getattr(node, "value", None), "id", "") == "mx_format_map":
                calls.append((node.lineno, ast.literal_eval(node.slice)))
        tables.sort()
        calls.sort()
        bs = None
        for node in ast.walk(fn):
            if isinstance(node, ast.Assign) and getattr(node.targets[0], "id", "") == "block_size":
                bs = ast.literal_eval(node.value)
        # element formats in call order (scale formats (8, 0) skipped)
        fmts = [c for _, c in calls if c != (8, 0)]
        kats[fn.name] = {
            "block_size": bs,
            "input": tables[0][1],
            "outputs": [{"format": list(f) if isinstance(f, tuple) else f, "expected": tab} for f, (_, tab) in zip(fmts, tables[1:])],
        }
    (OUT / "mx_kat.json").write_text(json.dumps(kats))


if __name__ == "__main__":
    steps = sys.argv[1:] or ["tensor_quant", "quantizer", "calib", "mtq_linear", "llama_fp8", "mixtral_fp8", "nvfp4", "export", "awq", "mse", "awq_clip", "kv", "presets", "mx_kat"]
    for s in steps:
        print("generating", s, flush=True)
        globals()["gen_" + s]()
    print("done")
