"""Shared helpers of the mtq.compress tests (goldens: tests/golden/make_golden_compress.py)."""

import copy
import json
from pathlib import Path

import torch
from safetensors.torch import load_file

G = Path(__file__).resolve().parent / "golden"
META = json.loads((G / "compress.json").read_text())
CASES = [c for c in META if c != "mxfp8_export"]


def tiny_llama_bf16():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=32, max_position_embeddings=64,
                      architectures=["LlamaForCausalLM"])
    torch.manual_seed(80)
    return LlamaForCausalLM(cfg).eval().to(torch.bfloat16)


def weight_only_cfg(mtq, preset, block):
    src = getattr(mtq, preset)
    w = copy.deepcopy(next(e for e in src["quant_cfg"] if e.get("quantizer_name") == "*weight_quantizer"))
    if block is not None:
        w["cfg"]["block_sizes"] = {-1: block, "type": "static"}
    return {"quant_cfg": [{"quantizer_name": "*", "enable": False}, w,
                          {"quantizer_name": "*lm_head*", "enable": False}], "algorithm": "max"}


def build(case, device, prefix=None):
    """The tiny Llama quantized as the reference's golden case, with the reference's
    post-calibration state loaded (weights + amax), not yet compressed."""
    import modelopt_amd.torch.quantization as mtq

    t = load_file(str(G / "compress.safetensors"))
    prefix = prefix or case
    preset, block = (META[case]["preset"], META[case]["block"]) if case in META and "preset" in META[case] \
        else ("MXFP8_DEFAULT_CFG", None)
    m = tiny_llama_bf16().to(device)
    ids = t["calib_ids"].to(device)
    mtq.quantize(m, weight_only_cfg(mtq, preset, block), lambda mm: [mm(b) for b in ids])
    state = {k[len(prefix) + 7:]: v for k, v in t.items() if k.startswith(prefix + ".state.")}
    missing, unexpected = m.load_state_dict(state, strict=False)
    assert not unexpected, unexpected
    assert not [k for k in missing if "quantizer" not in k], missing
    return m, t


def as_bytes(x):
    return x.view(torch.uint8) if x.element_size() == 1 else x


def check_compressed(case, m, t):
    """Packed bytes, scale buffers and dequantised weights bit-exact vs the reference."""
    from modelopt_amd.torch.quantization.qtensor import QTensorWrapper

    bad = []
    for n, info in META[case]["linears"].items():
        mod = m.get_submodule(n)
        w = mod.weight
        if not isinstance(w, QTensorWrapper) or w.metadata["qtensor_class"].__name__ != info["qtensor_class"]:
            bad.append((n, "not compressed"))
            continue
        if str(w.data.dtype) != info["qdtype"] or not torch.equal(as_bytes(w.data).cpu(), t[f"{case}.q.{n}"]):
            bad.append((n, "packed data"))
        for b in ("scale", "double_scale"):
            key = f"{case}.{b}.{n}"
            if key in t:
                got = getattr(mod.weight_quantizer, "_" + b)
                if not torch.equal(as_bytes(got).cpu().reshape(t[key].shape), t[key]) or got.dtype != (
                    torch.float8_e4m3fn if t[key].dtype == torch.uint8 and got.element_size() == 1 and got.dtype != torch.uint8 else got.dtype
                ):
                    bad.append((n, b))
        dq = mod.weight_quantizer(mod.weight)
        if not torch.equal(dq.cpu(), t[f"{case}.dq.{n}"]):
            bad.append((n, "dequantized weight"))
    return bad
