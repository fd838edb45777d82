"""Unified HF checkpoint export vs the reference's own export (tests/golden/export.*).

For each format the reference quantized a tiny Llama (hidden 64) on the CPU and exported it; the
golden holds its post-calibration state (weights + quantizer buffers) and the exported tensors
and configs.  Here the same model is converted with modelopt_amd, the reference's
post-calibration state is loaded (so calibration differences cannot leak in), and
export_hf_checkpoint must reproduce every exported tensor bit for bit and both JSON configs.
"""

import copy
import json
import os
from pathlib import Path

import pytest
import torch
from safetensors.torch import load_file

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"
META = json.loads((G / "export.json").read_text())


def _tiny():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=32, max_position_embeddings=64,
                      architectures=["LlamaForCausalLM"])
    torch.manual_seed(80)
    return LlamaForCausalLM(cfg).eval()


def _tiny_mixtral():
    from transformers import MixtralConfig, MixtralForCausalLM

    cfg = MixtralConfig(hidden_size=64, intermediate_size=64, num_hidden_layers=2, num_attention_heads=4,
                        num_key_value_heads=2, vocab_size=32, max_position_embeddings=64, num_local_experts=4,
                        num_experts_per_tok=2, architectures=["MixtralForCausalLM"])
    torch.manual_seed(82)
    return MixtralForCausalLM(cfg).eval()


def _cfg(mtq, preset):
    cfg = copy.deepcopy(getattr(mtq, preset))
    for e in cfg["quant_cfg"]:
        if e.get("quantizer_name") == "*weight_quantizer":
            c = e["cfg"]
            first = c[0] if isinstance(c, list) else c
            if first.get("num_bits") == 4:
                first["block_sizes"] = {-1: 32, "type": "static"}
            if first.get("num_bits") == (4, 3) and -2 in (first.get("block_sizes") or {}):
                first["block_sizes"] = {-1: 32, -2: 32}  # as make_golden.export_cfg
    return cfg


@pytest.mark.parametrize("case", sorted(META))
def test_export_matches_reference(gpu, case, tmp_path):
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.export import export_hf_checkpoint

    t = load_file(str(G / "export.safetensors"))
    ids = t["calib_ids"].to(gpu)
    model = (_tiny_mixtral() if META[case].get("model") == "mixtral" else _tiny()).to(gpu)
    mtq.quantize(model, _cfg(mtq, META[case]["preset"]), lambda m: [m(b) for b in ids])
    state = {k[len(case) + 7:]: v for k, v in t.items() if k.startswith(case + ".state.")}
    missing, unexpected = model.load_state_dict(state, strict=False)
    assert not unexpected, unexpected
    assert not [k for k in missing if "quantizer" not in k], missing
    export_hf_checkpoint(model, export_dir=str(tmp_path))
    got = load_file(str(tmp_path / "model.safetensors"))
    want = {k[len(case) + 8:]: v for k, v in t.items() if k.startswith(case + ".export.")}
    assert set(got) == set(want), (sorted(set(got) ^ set(want)))[:10]
    bad = []
    for k, v in want.items():
        g = got[k]
        if g.dtype != v.dtype or g.shape != v.shape:
            bad.append((k, g.dtype, v.dtype, tuple(g.shape), tuple(v.shape)))
        elif not torch.equal(g.view(torch.uint8) if g.element_size() == 1 else g, v.view(torch.uint8) if v.element_size() == 1 else v):
            bad.append((k, "values"))
    assert not bad, bad[:8]
    hq = json.loads((tmp_path / "hf_quant_config.json").read_text())
    hq["producer"]["version"] = None
    assert hq == META[case]["hf_quant_config"]
    cq = json.loads((tmp_path / "config.json").read_text())["quantization_config"]
    cq["producer"]["version"] = None
    assert cq == META[case]["quantization_config"]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("shape,block", [((256, 512), (128, 128)), ((200, 136), (64, 32)), ((64, 128), (32, 32)),
                                         ((1000, 1032), (128, 128))])
@pytest.mark.parametrize("scale_dtype", ["fp32", "own"])
def test_fp8_block2d_packer_matches_torch(gpu, dtype, shape, block, scale_dtype):
    """export_fp8_block2d (the FP8_PB_WO packer) against the reference expression
    (qtensor/fp8_tensor.py:60-117: pad, repeat_interleave the block scales, divide, cast) on the same
    device tensors: ragged edges, fp32 scales (fp32 quotient) and scales in the weight's own dtype
    (the quotient rounded to it), NaN / inf / overflowing elements."""
    from modelopt_amd import _ext

    ops = _ext.ops()
    g = torch.Generator(device=gpu).manual_seed(31)
    w = (torch.randn(shape, device=gpu, generator=g) * 3).to(dtype)
    w.view(-1)[7] = float("nan")
    w.view(-1)[11] = float("inf")
    w.view(-1)[13] = -1e4 if dtype != torch.float16 else -6e4  # overflows its block's scale
    br, bc = block
    nrb, ncb = -(-shape[0] // br), -(-shape[1] // bc)
    s = torch.rand(nrb, ncb, device=gpu, generator=g) * 0.02 + 1e-3
    if scale_dtype == "own":
        s = s.to(dtype)
    got = ops.export_fp8_block2d(w, s, br, bc)
    pad = torch.nn.functional.pad(w, (0, ncb * bc - shape[1], 0, nrb * br - shape[0]))
    exp = s.repeat_interleave(br, 0).repeat_interleave(bc, 1)
    want = (pad / exp).to(torch.float8_e4m3fn)[: shape[0], : shape[1]]
    gb, wb = got.view(torch.uint8), want.view(torch.uint8)
    nan = torch.isnan(got.float()) & torch.isnan(want.float())  # torch's NaN sign may differ (see exhaustive)
    assert bool(((gb == wb) | nan).all()), int((~((gb == wb) | nan)).sum())
