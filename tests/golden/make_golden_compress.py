#!/usr/bin/env python3
"""Goldens for mtq.compress (real-quant QTensors) and the MXFP8 unified export, from the REFERENCE
run on the CPU (same import shims as make_golden.py; run in the survey container only):

    python tests/golden/make_golden_compress.py

A tiny bf16 Llama (make_golden.tiny_llama_export) is calibrated per format with weight-only
quantizers, then ``modelopt.torch.quantization.compress`` packs every QuantLinear weight into a
QTensor (compress.py:196-225, tensor_quantizer.py:796-888).  Saved per case: the post-calibration
state dict, each compressed weight's packed bytes, its scale buffers (``_scale`` /
``_double_scale``), the dequantised weight (what the compressed model's forward uses) and the
logits of a test batch.  ``mxfp8_export``: export_hf_checkpoint of the MXFP8 model
(unified_export_hf.py:671-680).

Outputs: compress.safetensors / compress.json.
"""

from __future__ import annotations

import copy
import json
import os
import tempfile

import make_golden as mg  # noqa: F401  (installs the import shims, imports the reference)
import torch
from make_golden import OUT, mtq, save_file, tiny_llama_export

from modelopt.torch.quantization.qtensor import QTensorWrapper

CASES = {
    "fp8": ("FP8_DEFAULT_CFG", None),
    "int8": ("INT8_WEIGHT_ONLY_CFG", None),
    "int4": ("INT4_BLOCKWISE_WEIGHT_ONLY_CFG", 32),
    "nvfp4": ("NVFP4_DEFAULT_CFG", None),
    "mxfp4": ("MXFP4_DEFAULT_CFG", None),
    "mxfp8": ("MXFP8_DEFAULT_CFG", None),
}


def weight_only_cfg(preset: str, block: int | None):
    """The preset's weight quantizer alone (activation quantizers off: the MX / NVFP4 activation
    fake quant has no CPU path in the reference), lm_head off."""
    src = getattr(mtq, preset)
    w = next(e for e in src["quant_cfg"] if e.get("quantizer_name") == "*weight_quantizer")
    w = copy.deepcopy(w)
    if block is not None:
        w["cfg"]["block_sizes"] = {-1: block, "type": "static"}
    return {
        "quant_cfg": [
            {"quantizer_name": "*", "enable": False},
            w,
            {"quantizer_name": "*lm_head*", "enable": False},
        ],
        "algorithm": "max",
    }


def main():
    g = torch.Generator().manual_seed(91)
    ids = torch.randint(0, 32, (3, 2, 16), generator=g)
    test = torch.randint(0, 32, (2, 16), generator=g)
    t, meta = {"calib_ids": ids, "test_ids": test}, {}
    for name, (preset, block) in CASES.items():
        m = tiny_llama_export().to(torch.bfloat16)
        cfg = weight_only_cfg(preset, block)
        mtq.quantize(m, cfg, lambda mm: [mm(b) for b in ids])
        for k, v in m.state_dict().items():
            t[f"{name}.state.{k}"] = v.detach().clone().contiguous()
        mtq.compress(m)
        lin = {}
        for n, mod in m.named_modules():
            w = getattr(mod, "weight", None)
            if not isinstance(w, QTensorWrapper):
                continue
            data = w.data
            t[f"{name}.q.{n}"] = data.view(torch.uint8) if data.element_size() == 1 else data
            wq = mod.weight_quantizer
            for b in ("_scale", "_double_scale"):
                if getattr(wq, b, None) is not None:
                    v = getattr(wq, b)
                    t[f"{name}.{b[1:]}.{n}"] = v.view(torch.uint8) if v.dtype == torch.float8_e4m3fn else v
            t[f"{name}.dq.{n}"] = wq(mod.weight).detach()
            lin[n] = {"qtensor_class": w.metadata["qtensor_class"].__name__, "qdtype": str(data.dtype),
                      "shape": list(w.metadata["shape"])}
        with torch.no_grad():
            t[f"{name}.logits"] = m(test).logits.float()
        meta[name] = {"preset": preset, "block": block, "linears": lin}

    # MXFP8 unified export (unified_export_hf.py:671-680, quant_utils.py:309-310 / 871-872)
    from safetensors.torch import load_file

    from modelopt.torch.export import export_hf_checkpoint

    m = tiny_llama_export().to(torch.bfloat16)
    mtq.quantize(m, weight_only_cfg("MXFP8_DEFAULT_CFG", None), lambda mm: [mm(b) for b in ids])
    for k, v in m.state_dict().items():
        t[f"mxfp8_export.state.{k}"] = v.detach().clone().contiguous()
    with tempfile.TemporaryDirectory() as d:
        export_hf_checkpoint(m, export_dir=d)
        for k, v in load_file(os.path.join(d, "model.safetensors")).items():
            t[f"mxfp8_export.export.{k}"] = v.view(torch.uint8) if v.dtype == torch.float8_e4m3fn else v.contiguous()
        hq = json.load(open(os.path.join(d, "hf_quant_config.json")))
        cq = json.load(open(os.path.join(d, "config.json"))).get("quantization_config")
    hq["producer"]["version"] = None
    if cq and "producer" in cq:
        cq["producer"]["version"] = None
    meta["mxfp8_export"] = {"hf_quant_config": hq, "quantization_config": cq}
    save_file(t, str(OUT / "compress.safetensors"))
    (OUT / "compress.json").write_text(json.dumps(meta, indent=1))
    print("wrote", OUT / "compress.safetensors", len(t), "tensors")


if __name__ == "__main__":
    main()
