"""AWQ-lite DP exchanges keep every linear's result on that linear's device (a DP rank
whose model is spread over several devices by device_map).  `fixed_order_sum_many` packs the
tensors of all linears into one buffer on the first tensor's device; each slice must come back on
its own tensor's device, and `_awq_sync_act_scale` must leave act_scale beside the linear's
weight_scale (get_scale then builds the search tables on the weight's device).

One GPU box: the two "devices" are cuda:0 and the host, under a one-rank gloo group (the packed
path runs as it does at world N)."""

import os
import socket
import types

import pytest
import torch
import torch.distributed as dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def one_rank_group():
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        yield
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_fixed_order_sum_many_returns_each_slice_on_its_device(gpu, one_rank_group):
    from modelopt_amd.torch.utils.distributed import DistributedProcessGroup, fixed_order_sum_many

    a = torch.arange(6, dtype=torch.float32, device=gpu)
    b = torch.arange(4, dtype=torch.float32)
    out = fixed_order_sum_many([a, b], DistributedProcessGroup(None))
    assert out[0].device == a.device and out[1].device == b.device
    assert torch.equal(out[0].cpu(), a.cpu()) and torch.equal(out[1], b)


@pytest.mark.gpu
def test_awq_act_scale_stays_on_the_linear_device(gpu, one_rank_group):
    from modelopt_amd.torch.quantization import model_calib as mc
    from modelopt_amd.torch.utils.distributed import ParallelState

    mods = []
    for dev in (gpu, torch.device("cpu")):
        k = 8
        h = types.SimpleNamespace(num_cache_steps=2, act_scale=torch.full((k,), 4.0, device=dev),
                                  weight_scale=torch.ones(k, device=dev), is_enabled=True)
        m = types.SimpleNamespace(awq_lite=h, weight=torch.zeros(3, k, device=dev),
                                  parallel_state=ParallelState(data_parallel_group=None))
        mods.append((f"lin_{dev.type}", m))
    mc._awq_sync_act_scale(mods)
    for _, m in mods:
        h = m.awq_lite
        assert h.is_enabled
        assert h.act_scale.device == h.weight_scale.device
        assert torch.equal(h.act_scale.cpu(), torch.full((8,), 2.0))
