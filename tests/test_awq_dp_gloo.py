"""AWQ-lite data-parallel exchanges on CPU (gloo, world 2).

Reference model_calib.py:1595-1629 syncs every linear on its own: an ``all_gather_object`` of a NaN
flag and an ``all_reduce(AVG)`` of ``act_scale`` per linear (both gated on the rank-local
``num_cache_steps > 0``).  The product packs them: one fixed-order sum of all linears'
``[act_scale, nan, present]`` after the caching pass and one of all linears' losses after the
search pass (model_calib._awq_sync_act_scale / _awq_sync_losses).  Checked here:
* the number of collectives awq_lite issues does not depend on the number of linears;
* every rank ends with bit-identical scales and weights;
* a linear that receives tokens on one rank only (a sequential-MoE expert) neither hangs the
  group nor leaves the ranks with different decisions.
"""

import io
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

_CFG = {
    "quant_cfg": [
        {"quantizer_name": "*", "enable": False},
        {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4, "block_sizes": {-1: 8, "type": "static"}}},
    ],
    "algorithm": {"method": "awq_lite", "alpha_step": 0.1, "debug": True},
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Stack(nn.Module):
    def __init__(self, depth, skip_on_rank1=False):
        super().__init__()
        torch.manual_seed(3)
        self.layers = nn.ModuleList(nn.Linear(16, 16) for _ in range(depth))
        self.expert = nn.Linear(16, 16)
        self.skip_on_rank1 = skip_on_rank1

    def forward(self, x):
        for lin in self.layers:
            x = torch.relu(lin(x))
        if not (self.skip_on_rank1 and dist.get_rank() == 1):
            x = x + self.expert(x)  # an expert that only rank 0 routes tokens to
        return x


def _count_collectives(fn):
    names = ["all_gather", "all_reduce", "all_gather_object", "broadcast", "all_gather_into_tensor",
             "reduce_scatter", "broadcast_object_list"]
    saved = {n: getattr(dist, n) for n in names}
    count = [0]

    def wrap(f):
        def w(*a, **k):
            count[0] += 1
            return f(*a, **k)
        return w

    for n, f in saved.items():
        setattr(dist, n, wrap(f))
    try:
        fn()
    finally:
        for n, f in saved.items():
            setattr(dist, n, f)
    return count[0]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import modelopt_amd.torch.quantization as mtq

        g = torch.Generator().manual_seed(50 + rank)
        data = [torch.randn(4, 16, generator=g) for _ in range(2)]
        res = {}
        for depth in (2, 6):
            model = _Stack(depth)
            n = _count_collectives(lambda: mtq.quantize(model, _CFG, lambda m: [m(d) for d in data]))
            res[depth] = (n, {k: v.detach().clone() for k, v in model.state_dict().items() if k.endswith("weight")})
        moe = _Stack(2, skip_on_rank1=True)
        mtq.quantize(moe, _CFG, lambda m: [m(d) for d in data])
        res["moe"] = (0, {k: v.detach().clone() for k, v in moe.state_dict().items() if k.endswith("weight")})
        res["moe_enabled"] = bool(moe.expert.awq_lite.is_enabled)
        buf = io.BytesIO()  # plain bytes: tensors on a Queue die with the sending process
        torch.save(res, buf)
        q.put((rank, buf.getvalue()))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_awq_lite_packed_dp_exchange_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=200) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in out.values():
        assert not isinstance(r, str), r
    r0, r1 = (torch.load(io.BytesIO(out[i]), weights_only=True) for i in (0, 1))
    # constant number of collectives (max calibration's packed MAX + two AWQ packs), whatever the depth
    assert r0[2][0] == r0[6][0] == r1[2][0] == r1[6][0], (r0[2][0], r0[6][0])
    assert r0[2][0] <= 4
    for key in (2, 6, "moe"):
        w0, w1 = r0[key][1], r1[key][1]
        assert w0.keys() == w1.keys()
        for k in w0:
            assert torch.equal(w0[k], w1[k]), (key, k)
    assert r0["moe_enabled"] == r1["moe_enabled"] is True
