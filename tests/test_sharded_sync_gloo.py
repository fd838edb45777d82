"""``sync_sharded_amax`` beyond amax: after layer-sharded calibration the owner's
``_pre_quant_scale`` (AWQ / SmoothQuant) and the NVFP4 static weight quantizers' block amax must
reach every rank in the one packed exchange, the NVFP4 global amax must be re-derived on every rank
by the promotion (max of the block amax, reference core_utils.py:1129-1143), and a non-owner that
still holds real weights must be refused (the owner folded 1/s into its own weights).  gloo, world 2.
"""

import io
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

_NVFP4_W = {
    "quant_cfg": [
        {"quantizer_name": "*", "enable": False},
        {"quantizer_name": "*weight_quantizer",
         "cfg": {"num_bits": (2, 1), "block_sizes": {-1: 16, "type": "static", "scale_bits": (4, 3)}}},
        {"quantizer_name": "*input_quantizer", "cfg": {"num_bits": 8, "axis": None}},
    ],
    "algorithm": "max",
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(4)
    return nn.Sequential(nn.Linear(32, 32), nn.Linear(32, 32))


def _state(model):
    out = {}
    for n, m in model.named_modules():
        for attr in ("_amax", "_pre_quant_scale", "_global_amax"):
            v = m.__dict__.get("_buffers", {}).get(attr)
            if isinstance(v, torch.Tensor) and v.device.type != "meta":
                out[f"{n}.{attr}"] = v.detach().clone()
    return out


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import modelopt_amd.torch.quantization as mtq
        from modelopt_amd.torch.quantization.nn.modules import quant_module as qm
        from modelopt_amd.torch.quantization.sharded import sync_sharded_amax

        prev, qm._DEFAULT_DP_GROUP = qm._DEFAULT_DP_GROUP, -1
        try:
            full = mtq.quantize(_model(), _NVFP4_W, lambda m: m(torch.randn(4, 32)))
            for i, lin in enumerate(full):
                lin.input_quantizer.pre_quant_scale = torch.rand(32) + 0.5 + i
            want = _state(full)
            # sharded: rank r owns layer r; the other layer's params and quantizer state on meta
            model = mtq.quantize(_model(), _NVFP4_W, lambda m: m(torch.randn(4, 32)))
        finally:
            qm._DEFAULT_DP_GROUP = prev
        other = model[1 - rank]
        other.to("meta")
        for n, m in other.named_modules():
            for attr in ("_amax", "_pre_quant_scale", "_global_amax"):
                if attr in getattr(m, "_buffers", {}):
                    del m._buffers[attr]
        own, ref = model[rank], full[rank]
        own.weight_quantizer.amax = ref.weight_quantizer._amax.clone()
        own.input_quantizer.amax = ref.input_quantizer._amax.clone()
        own.input_quantizer.pre_quant_scale = ref.input_quantizer._pre_quant_scale.clone()
        sync_sharded_amax(model, device=torch.device("cpu"))
        got = _state(model)
        # a non-owner with real weights is refused
        refused = False
        real = _model()
        qm._DEFAULT_DP_GROUP = -1
        try:
            real = mtq.quantize(real, _NVFP4_W, lambda m: m(torch.randn(4, 32)))
        finally:
            qm._DEFAULT_DP_GROUP = prev
        for lin in real:
            if "_pre_quant_scale" in lin.input_quantizer._buffers:
                del lin.input_quantizer._buffers["_pre_quant_scale"]
        real[rank].input_quantizer.pre_quant_scale = torch.ones(32)
        try:
            sync_sharded_amax(real, device=torch.device("cpu"))
        except RuntimeError:
            refused = True
        buf = io.BytesIO()
        torch.save({"want": want, "got": got, "refused": refused}, buf)
        q.put((rank, buf.getvalue()))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_sync_pre_quant_scale_and_nvfp4_global_amax_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in out.values():
        assert not isinstance(r, str), r
    for rank in range(world):
        d = torch.load(io.BytesIO(out[rank]), weights_only=True)
        want, got = d["want"], d["got"]
        # every quantizer tensor the single process holds, on every rank, bit for bit
        for k, v in want.items():
            assert k in got, (rank, k)
            assert torch.equal(got[k].float(), v.float()), (rank, k)
        assert any(k.endswith("_pre_quant_scale") for k in want)
        assert any(k.endswith("_global_amax") for k in want), sorted(want)
        assert d["refused"], rank
