"""Layer-sharded (pipelined) calibration machinery on CPU with gloo.

Each rank owns a contiguous stage of decoder layers (the others are moved to the meta device, so
any compute outside the stage would fail); the owned layers must see exactly the hidden states a
single-process whole-model forward gives them, and ``sync_sharded_amax`` must leave every rank
with every quantizer's amax after one packed all-reduce."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from modelopt_amd.torch.quantization.sharded import layer_shard_plan


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tiny_llama(layers):
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=32, intermediate_size=64, num_hidden_layers=layers, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=50, max_position_embeddings=64)
    torch.manual_seed(0)
    return LlamaForCausalLM(cfg).eval()


def _record(layers, idxs, store):
    """Hidden states entering each layer's compute (its input_layernorm), i.e. after the stage's
    receive substitution."""
    hs = []
    for i in idxs:
        store[i] = []
        hs.append(layers[i].input_layernorm.register_forward_pre_hook(
            lambda m, a, i=i: store[i].append(a[0].clone())))
    return hs


def _worker(rank, world, port, nlayers, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import modelopt_amd.torch.quantization as mtq
        from modelopt_amd.torch.quantization.sharded import layer_sharded_calibration, sync_sharded_amax

        model = _tiny_llama(nlayers)
        layers = model.model.layers
        g = torch.Generator().manual_seed(5)
        batches = [torch.randint(0, 50, (2, 10), generator=g) for _ in range(3)]
        want = {}
        hs = _record(layers, range(nlayers), want)
        with torch.no_grad():
            ref_logits = [model(b).logits for b in batches]
        for h in hs:
            h.remove()

        plan = layer_shard_plan(nlayers, rank, world)
        for i in range(nlayers):
            if i not in plan.owned:
                layers[i].to("meta")
        if rank != world - 1:
            model.lm_head.to("meta")
        got = {}
        hs = _record(layers, plan.owned, got)
        outs = []
        with layer_sharded_calibration(model, plan), torch.no_grad():
            for b in batches:
                outs.append(model(b))
        for h in hs:
            h.remove()
        ok_inputs = all(
            len(got[i]) == len(batches) and all(torch.equal(a, b) for a, b in zip(got[i], want[i]))
            for i in plan.owned
        )
        if rank == world - 1:
            ok_out = all(torch.allclose(o.logits, r, rtol=0, atol=0) for o, r in zip(outs, ref_logits))
        else:
            ok_out = all(o is None for o in outs)

        # amax exchange: owners hold values (per-tensor and per-channel), others meta / nothing
        mtq.conversion.replace_quant_module(model)
        expect = {}
        for name, m in model.named_modules():
            if isinstance(m, mtq.TensorQuantizer) and ".layers." in name:
                li = int(name.split(".layers.")[1].split(".")[0])
                shape = (7, 1) if name.endswith("weight_quantizer") else ()
                val = torch.full(shape, float(li * 100 + len(name)))
                expect[name] = val
                if li in plan.owned:
                    m.amax = val
                elif name.endswith("weight_quantizer"):
                    m.amax = torch.empty(shape, device="meta")
        n = sync_sharded_amax(model, device=torch.device("cpu"))
        mods = dict(model.named_modules())
        ok_amax = all(torch.equal(mods[k].amax, v) for k, v in expect.items())
        q.put((rank, ok_inputs, ok_out, ok_amax, n, sum(v.numel() for v in expect.values())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nlayers", [(2, 4), (3, 4)])
@pytest.mark.timeout(180)
def test_layer_sharded_pipeline(world, nlayers):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nlayers, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs)
    for rank, ok_inputs, ok_out, ok_amax, n, total in res:
        assert ok_inputs, f"rank {rank}: stage inputs differ from the whole-model forward"
        assert ok_out, f"rank {rank}: outputs"
        assert ok_amax and n == total, f"rank {rank}: amax exchange ({n} vs {total})"


def test_shard_plan_balanced():
    plans = [layer_shard_plan(80, r, 8) for r in range(8)]
    assert [p.first for p in plans] == list(range(0, 80, 10)) and plans[-1].last == 80
    plans = [layer_shard_plan(10, r, 4) for r in range(4)]
    assert [(p.first, p.last) for p in plans] == [(0, 3), (3, 6), (6, 8), (8, 10)]


def test_sender_keeps_one_send_in_flight(monkeypatch):
    """The stage hand-off is a non-blocking isend: the next send (or the context exit) first waits
    for the previous transfer, and the sent tensor is held until that wait returns."""
    import modelopt_amd.torch.quantization.sharded as sh

    log = []

    class _Work:
        def __init__(self, i):
            self.i = i

        def wait(self):
            log.append(("wait", self.i))

    def fake_isend(t, dst, group):
        log.append(("isend", int(t[0]), dst))
        return _Work(int(t[0]))

    monkeypatch.setattr(sh.dist, "isend", fake_isend)
    monkeypatch.setattr(sh, "_is_gloo", lambda g: True)
    s = sh._Sender()
    s.send(torch.tensor([1.0]), 1, None)
    assert log == [("isend", 1, 1)] and s._tensor is not None
    s.send(torch.tensor([2.0]), 1, None)
    assert log == [("isend", 1, 1), ("wait", 1), ("isend", 2, 1)]
    s.wait()
    assert log[-1] == ("wait", 2) and s._tensor is None and s._work is None
