"""Data-parallel calibration end to end: ``mtq.quantize`` on 2 ranks (gloo, sharing the one MI355X)
with the calibration samples split across the ranks, against a single process over all samples.

* FP8 ``max`` on a tiny Llama: the packed amax ``all_reduce(MAX)`` (model_calib.sync_amax_packed;
  reference model_calib.py:390-407 / tensor_quantizer.py:1373-1385, one collective per quantizer)
  gives every rank the single-process amax bit for bit (max is exact and order-free).
* ``awq_lite`` (INT4 block 8) on the reference test MLP: ``act_scale`` is averaged over the ranks
  by a fixed-order fp32 sum (utils/distributed.fixed_order_sum; reference :1588-1593 uses
  all_reduce(AVG)) and the per-alpha losses are summed the same way, so all ranks end with
  bit-identical scales and weights.  Against the single process: same best alpha per layer,
  act_scale within rtol 1e-6 (per-rank means averaged vs one mean over all batches: the two fp32
  summation orders differ by a few ulp), best scales within rtol 1e-5.
Reference multi-process test: tests/unit/torch/quantization/test_dist.py:27-47.
"""

from __future__ import annotations

import io
import os
import socket

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tiny_llama():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=64, max_position_embeddings=128)
    torch.manual_seed(0)
    return LlamaForCausalLM(cfg).eval().to(torch.bfloat16)


class _SimpleMLP(nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(1)
        self.net = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 16), nn.ReLU(), nn.Linear(16, 16))

    def forward(self, x):
        return self.net(x)


_AWQ_CFG = {
    "quant_cfg": [
        {"quantizer_name": "*", "enable": False},
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4, "block_sizes": {-1: 8, "type": "static"}}},
    ],
    "algorithm": {"method": "awq_lite", "alpha_step": 0.1, "debug": True},
}


def _run(kind, data, dev):
    import modelopt_amd.torch.quantization as mtq

    def loop(m):
        with torch.no_grad():
            for d in data:
                m(d.to(dev))

    if kind == "fp8":
        model = mtq.quantize(_tiny_llama().to(dev), mtq.FP8_DEFAULT_CFG, loop)
        return {n: m.amax.detach().cpu() for n, m in model.named_modules()
                if isinstance(m, mtq.TensorQuantizer) and m.amax is not None}
    model = mtq.quantize(_SimpleMLP().to(dev), _AWQ_CFG, loop)
    res = {}
    for n, m in model.named_modules():
        if hasattr(m, "awq_lite"):
            h = m.awq_lite
            res[n] = {"alpha": h.best_alpha, "act_scale": h.act_scale.detach().cpu(),
                      "scale": h.best_scale.detach().cpu(), "weight": m.weight.detach().cpu()}
    return res


def _data(kind):
    g = torch.Generator().manual_seed(11)
    if kind == "fp8":
        return [torch.randint(0, 64, (2, 16), generator=g) for _ in range(4)]
    return [torch.randn(8, 16, generator=g) for _ in range(4)]


def _worker(rank, world, port, kind, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        data = _data(kind)
        mine = data[rank::world]
        dp = _run(kind, mine, dev)
        # the single-process reference, with the default group disabled for these modules
        from modelopt_amd.torch.quantization.nn.modules import quant_module as qm

        prev, qm._DEFAULT_DP_GROUP = qm._DEFAULT_DP_GROUP, -1
        try:
            single = _run(kind, data, dev)
        finally:
            qm._DEFAULT_DP_GROUP = prev
        buf = io.BytesIO()  # plain bytes: tensors on a Queue die with the sending process
        torch.save({"dp": dp, "single": single}, buf)
        q.put((rank, buf.getvalue(), None))
    except Exception as e:
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def _spawn(kind, world=2):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert not isinstance(r[1], str), r[1]
    assert all(p.exitcode == 0 for p in procs)
    out = []
    for rank, blob, _ in res:
        d = torch.load(io.BytesIO(blob), weights_only=True)
        out.append((rank, d["dp"], d["single"]))
    return out


@pytest.mark.timeout(300)
def test_dp_max_calibration_matches_single_process(gpu):
    res = _spawn("fp8")
    for rank, dp, single in res:
        assert set(dp) == set(single) and len(dp) > 0
        for k, v in single.items():
            assert torch.equal(dp[k], v), (rank, k)


@pytest.mark.timeout(300)
def test_dp_awq_lite_deterministic_and_matches_single_process(gpu):
    res = _spawn("awq")
    (_, dp0, single), (_, dp1, _) = res
    assert set(dp0) == set(single) and len(dp0) == 3
    for n in single:
        for key in ("act_scale", "scale", "weight"):  # every rank: the same bits
            assert torch.equal(dp0[n][key], dp1[n][key]), (n, key)
        assert dp0[n]["alpha"] == dp1[n]["alpha"] == single[n]["alpha"], n
        torch.testing.assert_close(dp0[n]["act_scale"], single[n]["act_scale"], rtol=1e-6, atol=0)
        torch.testing.assert_close(dp0[n]["scale"], single[n]["scale"], rtol=1e-5, atol=0)
