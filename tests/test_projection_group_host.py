"""Host side of the grouped q/k/v decode projections (quant_linear.ProjectionGroup, installed by
the HF attention wrapper): on inputs the fused kernels do not take (CPU tensors here) every
projection runs its own reference path, each input quantizer once, and the wrapper removes the
group after the forward."""

import torch


def test_projection_group_installed_and_inert_on_cpu():
    from transformers import LlamaConfig, LlamaForCausalLM

    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.nn.modules import quant_linear as ql

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=1, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=64, max_position_embeddings=32)
    torch.manual_seed(1)
    model = LlamaForCausalLM(cfg).eval()
    ids = torch.randint(0, 64, (2, 8))
    mtq.quantize(model, mtq.FP8_DEFAULT_CFG, lambda m: m(ids))
    attn = model.model.layers[0].self_attn
    projs = attn._qkv_projections()
    assert [p is getattr(attn, n) for p, n in zip(projs, ("q_proj", "k_proj", "v_proj"))] == [True] * 3
    seen = []
    real = ql.ProjectionGroup.take

    def spy(self, mod, inp):
        seen.append(mod)
        return real(self, mod, inp)

    ql.ProjectionGroup.take = spy
    try:
        with torch.no_grad():
            out = model(ids[:1, :1]).logits
    finally:
        ql.ProjectionGroup.take = real
    assert seen == projs  # each projection asked once, none served from the group on the CPU
    assert torch.isfinite(out).all()
    assert all("_projection_group" not in p.__dict__ for p in projs)
