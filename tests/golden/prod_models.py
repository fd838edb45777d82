"""Production-shape models of the E2E goldens (tests/golden/prod.*): built in fp32 on the CPU from
a seed and cast to bf16, so the generator (make_golden.py, reference on the CPU) and the GPU test
(tests/test_gpu_prod_e2e.py) hold the same weights; their sha256 fingerprint pins that."""

from __future__ import annotations

import hashlib

import torch

PROD_LLAMA = dict(hidden_size=4096, intermediate_size=14336, num_hidden_layers=2, num_attention_heads=32,
                  num_key_value_heads=8, vocab_size=512, max_position_embeddings=256, rope_theta=500000.0,
                  rms_norm_eps=1e-5)
PROD_MIXTRAL = dict(hidden_size=1024, intermediate_size=3584, num_hidden_layers=1, num_attention_heads=8,
                    num_key_value_heads=2, vocab_size=512, max_position_embeddings=256, num_local_experts=8,
                    num_experts_per_tok=2, rope_theta=1e6, rms_norm_eps=1e-5)
# name -> (model kind, seed, preset, algorithm override)
PROD_CASES = {
    "llama_fp8": ("llama", 80, "FP8_DEFAULT_CFG", None),
    "llama_int8": ("llama", 80, "INT8_DEFAULT_CFG", None),
    "llama_int4_awq": ("llama", 80, "INT4_AWQ_CFG", {"method": "awq_lite", "alpha_step": 0.1, "debug": True}),
    "mixtral_fp8": ("mixtral", 90, "FP8_DEFAULT_CFG", None),
}


def sha(t: torch.Tensor) -> str:
    t = t.detach().contiguous().cpu()
    return hashlib.sha256(t.view(torch.uint8).numpy().tobytes() if t.numel() else b"").hexdigest()


def fingerprint(model) -> dict:
    return {k: sha(v) for k, v in model.state_dict().items()}


def prod_model(kind: str, seed: int):
    """Llama-3-8B layer shapes (2 layers) / one Mixtral layer at hidden 1024 with 8 experts."""
    from transformers import LlamaConfig, LlamaForCausalLM, MixtralConfig, MixtralForCausalLM

    if kind == "llama":
        cfg, cls = LlamaConfig(**PROD_LLAMA), LlamaForCausalLM
    else:
        cfg, cls = MixtralConfig(**PROD_MIXTRAL), MixtralForCausalLM
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(seed)
    m = cls(cfg).eval().to(torch.bfloat16)
    if kind == "mixtral":
        m.config._experts_implementation = "eager"
    return m


def prod_inputs(seed: int):
    g = torch.Generator().manual_seed(seed + 1)
    ids = torch.randint(0, 512, (2, 2, 48), generator=g)
    test = torch.randint(0, 512, (1, 32), generator=g)
    return ids, test
