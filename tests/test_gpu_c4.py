"""Config C4 on the GPU: MXFP4 (E2M1 elements, block 32, E8M0 scales) weight + activation PTQ of
a Llama-architecture model, and its layer-sharded calibration across ranks.

* ``test_c4_tiny_llama_mxfp4_every_qdq_bit_exact``: ``mtq.quantize(tiny LlamaForCausalLM,
  MXFP4_DEFAULT_CFG + max)``; every enabled quantizer's fake-quantized tensor in the quantized
  forward equals ``oracle.fused_amax_convert(x, 32, "E2M1")`` (KAT-pinned, tests/golden/mx_kat.json)
  bit for bit, and every collected amax equals the exact max of |x| over the calibration inputs
  that quantizer saw.  Reference: tensor_quant.py:157-195 (dynamic block qdq), tensor_quant_mx.cu
  :240-387, calib/max.py (amax collection).
* ``test_c4_layer_sharded_two_ranks_share_one_gpu``: the layer-sharded pipeline of
  ``sharded.py`` (C4's 8-GPU plan) as 2 processes on the one MI355X, gloo backend (hidden states
  and the packed amax all-reduce host-staged): every rank's final amax state and the last stage's
  quantized logits equal a single-process run exactly, with a non-empty packed exchange.
  Reference: model_calib.py:2051-2189 (layerwise calibration), tensor_quantizer.py:1373-1385.
"""

from __future__ import annotations

import os
import socket

import pytest
import torch

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu


def _tiny_llama(layers=4, seed=0):
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=layers, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=64, max_position_embeddings=128)
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(seed)
    return LlamaForCausalLM(cfg).eval().to(torch.bfloat16)


def _cfg():
    import modelopt_amd.torch.quantization as mtq

    return {**mtq.MXFP4_DEFAULT_CFG, "algorithm": "max"}


def _batches(n=3, seed=5):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, 64, (4, 24), generator=g) for _ in range(n)]


def test_c4_tiny_llama_mxfp4_every_qdq_bit_exact(gpu):
    import modelopt_amd.torch.quantization as mtq

    model = _tiny_llama().to(gpu)
    batches = [b.to(gpu) for b in _batches()]
    seen: dict[str, torch.Tensor] = {}

    def calib_hook(name):
        def h(mod, inp, out):
            a = inp[0].detach().float().abs().amax()
            seen[name] = torch.maximum(seen[name], a) if name in seen else a
        return h

    def loop(m):
        with torch.no_grad():
            for b in batches:
                m(b)

    # register the calibration hooks once the quantizers exist (conversion runs inside quantize)
    model = mtq.quantize(model, _cfg(), lambda m: None)  # convert + (empty) calibrate
    qs = {n: q for n, q in model.named_modules() if isinstance(q, mtq.TensorQuantizer) and q.is_enabled}
    assert len(qs) == 2 * 7 * 4, "q/k/v/o/gate/up/down x (input, weight) x 4 layers"
    for q in qs.values():
        q.reset_amax()
    hs = [q.register_forward_hook(calib_hook(n)) for n, q in qs.items()]
    mtq.calibrate(model, "max", loop)
    for h in hs:
        h.remove()
    for n, q in qs.items():
        # MX quantizers keep the collected amax in _amax; their `amax` property reads None
        # (the scales are dynamic), as in the reference (tensor_quantizer.py amax property)
        a = getattr(q, "_amax", None)
        assert a is not None and q.amax is None, n
        assert torch.equal(a.detach().float().reshape(()).cpu(), seen[n].cpu()), n

    captured = []
    hs = [q.register_forward_hook(lambda m, i, o, n=n: captured.append((n, i[0].detach(), o.detach())))
          for n, q in qs.items()]
    with torch.no_grad():
        model(batches[0])
    for h in hs:
        h.remove()
    assert {n for n, _, _ in captured} == set(qs)
    for n, x, y in captured:
        ref = R.fused_amax_convert(x.cpu(), 32, "E2M1")
        got = y.cpu()
        assert got.dtype == ref.dtype == torch.bfloat16, n
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16)), n


# ---------------------------------------------------------------------------------------------
# layer-sharded C4 pipeline, 2 ranks on one GPU
# ---------------------------------------------------------------------------------------------


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_worker(rank, world, port, nlayers, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import modelopt_amd.torch.quantization as mtq
        from modelopt_amd.torch.quantization.sharded import (
            layer_shard_plan,
            layer_sharded_calibration,
            sync_sharded_amax,
        )

        dev = torch.device("cuda", 0)
        batches = [b.to(dev) for b in _batches()]
        test_ids = _batches(1, seed=9)[0].to(dev)

        def loop(m):
            with torch.no_grad():
                for b in batches:
                    m(b)

        # single-process reference (whole model on this rank)
        full = mtq.quantize(_tiny_llama(nlayers).to(dev), _cfg(), loop)
        ref_amax = {n: m._amax.detach().cpu() for n, m in full.named_modules()
                    if isinstance(m, mtq.TensorQuantizer) and getattr(m, "_amax", None) is not None}
        with torch.no_grad():
            ref_logits = full(test_ids).logits.cpu()
        del full

        model = _tiny_llama(nlayers).to(dev)
        plan = layer_shard_plan(nlayers, rank, world)
        for i in range(nlayers):
            if i not in plan.owned:
                model.model.layers[i].to("meta")
        if rank != world - 1:
            model.lm_head.to("meta")
        with layer_sharded_calibration(model, plan):
            mtq.quantize(model, _cfg(), loop)
        n = sync_sharded_amax(model, device=dev)
        got = {nm: m._amax.detach().cpu() for nm, m in model.named_modules()
               if isinstance(m, mtq.TensorQuantizer) and getattr(m, "_amax", None) is not None
               and not m._amax.is_meta}
        ok_amax = set(got) == set(ref_amax) and all(torch.equal(got[k], v) for k, v in ref_amax.items())
        with layer_sharded_calibration(model, plan), torch.no_grad():
            out = model(test_ids)
        if rank == world - 1:
            ok_logits = torch.equal(out.logits.cpu(), ref_logits)
        else:
            ok_logits = out is None
        q.put((rank, ok_amax, ok_logits, n, len(ref_amax), sorted(set(ref_amax) ^ set(got))[:4]))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, False, False, -1, 0, [repr(e)]))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_c4_layer_sharded_two_ranks_share_one_gpu(gpu):
    import torch.multiprocessing as mp

    world, nlayers = 2, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, nlayers, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, ok_amax, ok_logits, n, n_q, diff in res:
        assert ok_amax, f"rank {rank}: amax state differs from the single-process run {diff}"
        assert ok_logits, f"rank {rank}: last-stage logits differ"
        assert n >= n_q > 0, f"rank {rank}: packed exchange {n} entries for {n_q} quantizers"
