"""Multi-process amax exchange on CPU (gloo, world_size 2) -- the N>1 calibration path.

Reference: tests/unit/torch/quantization/test_dist.py:27-47 (DDP amax MAX check).  Here the packed
single-collective sync (model_calib.sync_amax_packed) must equal the per-quantizer MAX all-reduce.
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from modelopt_amd.torch.quantization.config import QuantizerAttributeConfig
        from modelopt_amd.torch.quantization.model_calib import sync_amax_packed
        from modelopt_amd.torch.quantization.nn import TensorQuantizer
        from modelopt_amd.torch.utils.distributed import DistributedProcessGroup

        g = torch.Generator().manual_seed(100 + rank)
        qs = []
        for shape, dt in [((), torch.bfloat16), ((8, 1), torch.float32), ((5,), torch.float16), ((3, 1), torch.float32)]:
            tq = TensorQuantizer(QuantizerAttributeConfig(num_bits=8))
            tq.amax = (torch.rand(shape, generator=g) * (rank + 1)).to(dt)
            qs.append(tq)
        nocal = TensorQuantizer()  # no amax: skipped
        before = [t.amax.clone() for t in qs]
        n = sync_amax_packed(qs + [nocal], DistributedProcessGroup(None))
        # reference semantics: one all_reduce(MAX) per quantizer
        ref = []
        for b in before:
            r = b.clone().float()
            dist.all_reduce(r, op=dist.ReduceOp.MAX)
            ref.append(r.to(b.dtype))
        ok = all(torch.equal(t.amax, r) for t, r in zip(qs, ref))
        q.put((rank, n, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_packed_amax_sync_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs)
    for rank, n, ok in res:
        assert n == 1, "one collective for all quantizers"
        assert ok, f"rank {rank}: packed sync != per-quantizer MAX all-reduce"


def _sum_worker(rank, world, port, q):
    import torch.distributed as dist

    from modelopt_amd.torch.utils.distributed import DistributedProcessGroup, fixed_order_sum

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(100 + rank)
        t = torch.randn(4096, generator=g) * 10 ** torch.randint(-6, 6, (4096,), generator=g).float()
        got = fixed_order_sum(t, DistributedProcessGroup(None))
        # the same rank-order sum computed from every rank's tensor regenerated locally
        parts = []
        for r in range(world):
            gr = torch.Generator().manual_seed(100 + r)
            parts.append(torch.randn(4096, generator=gr) * 10 ** torch.randint(-6, 6, (4096,), generator=gr).float())
        want = parts[0].clone()
        for p in parts[1:]:
            want += p
        q.put((rank, bool(torch.equal(got, want)), got.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_fixed_order_sum_world3_identical_bits():
    """utils.distributed.fixed_order_sum (AWQ act_scale / loss DP reduction, replacing the
    reference's all_reduce(AVG), model_calib.py:1588-1593): the rank-order fp32 sum on every rank,
    bit-identical across ranks (gloo has no AVG; RCCL's ring order is not fixed)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sum_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(3)]
    for p in procs:
        p.join(timeout=30)
    assert all(ok for _, ok, _ in res)
    assert len({b for _, _, b in res}) == 1
