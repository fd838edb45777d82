"""The RCCL ("nccl" backend) code paths on the MI355X at world size 1.

Every other multi-process GPU test initialises ``gloo`` (two ranks cannot share one GPU under
RCCL), so the device-tensor branches of the product's collectives only run here:

* (a) ``max_calibrate``'s packed ``all_reduce(MAX)`` on a device buffer
  (``model_calib.sync_amax_packed``; reference tensor_quantizer.py:1373-1385, model_calib.py:390-407);
* (b) AWQ-lite's ``fixed_order_sum_many`` -> ``all_gather`` of device tensors
  (``utils/distributed.py`` ``fixed_order_sum``; reference model_calib.py:1588-1593), on the fp32
  reference MLP and on a bf16 block-128 MLP that takes the fused search fast path;
* (c) ``layer_sharded_calibration`` with the world-1 plan, then ``sync_sharded_amax``: the layout
  ``all_gather_object`` and the packed device ``all_reduce(MAX)`` (``sharded.py``);
* (d) ``bench.py --gpus 1`` under a child ``torch.distributed.run --nproc-per-node=1``: its
  ``init_process_group("nccl", device_id=...)`` and the device max-over-ranks.

One child process (spawned before it touches the GPU) initialises ``nccl`` with rank 0 / world 1
and runs (a)-(c) twice: with the world group as the data-parallel group, and with the group
disabled (the no-dist run).  A spy on ``torch.distributed`` records every collective's backend and
tensor device, so the test fails if a path silently took a host-staged branch.  Every amax, AWQ
scale / weight and logit must be bit-equal between the two runs.  The point-to-point hand-off of
``sharded.py`` (``isend`` / ``recv`` between stages) has no peer at world 1 and stays unexecuted
until an 8-GPU node.
"""

from __future__ import annotations

import io
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tiny_llama(layers=2):
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=layers, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=64, max_position_embeddings=128)
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(0)
    return LlamaForCausalLM(cfg).eval().to(torch.bfloat16)


class _MLP(nn.Module):
    def __init__(self, dims, dtype, seed):
        super().__init__()
        torch.manual_seed(seed)
        layers = []
        for i in range(len(dims) - 1):
            layers += [nn.Linear(dims[i], dims[i + 1]), nn.ReLU()]
        self.net = nn.Sequential(*layers[:-1]).to(dtype)

    def forward(self, x):
        return self.net(x)


def _awq_cfg(block):
    return {
        "quant_cfg": [
            {"quantizer_name": "*", "enable": False},
            {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4, "block_sizes": {-1: block, "type": "static"}}},
        ],
        "algorithm": {"method": "awq_lite", "alpha_step": 0.1, "debug": True},
    }


def _amax_state(model, mtq):
    return {n: m._amax.detach().cpu() for n, m in model.named_modules()
            if isinstance(m, mtq.TensorQuantizer) and getattr(m, "_amax", None) is not None
            and not m._amax.is_meta}


def _case_fp8(dev, mtq):
    g = torch.Generator().manual_seed(11)
    batches = [torch.randint(0, 64, (2, 16), generator=g).to(dev) for _ in range(4)]
    ids = torch.randint(0, 64, (2, 16), generator=g).to(dev)

    def loop(m):
        with torch.no_grad():
            for b in batches:
                m(b)

    model = mtq.quantize(_tiny_llama().to(dev), mtq.FP8_DEFAULT_CFG, loop)
    with torch.no_grad():
        logits = model(ids).logits.cpu()
    return {"amax": _amax_state(model, mtq), "logits": logits}


def _case_awq(dev, mtq, dims, dtype, block, tokens):
    g = torch.Generator().manual_seed(12)
    data = [torch.randn(tokens, dims[0], generator=g).to(dev, dtype) for _ in range(3)]

    def loop(m):
        with torch.no_grad():
            for d in data:
                m(d)

    model = mtq.quantize(_MLP(dims, dtype, seed=3).to(dev), _awq_cfg(block), loop)
    res = {}
    for n, m in model.named_modules():
        if hasattr(m, "awq_lite"):
            h = m.awq_lite
            res[n] = {"alpha": torch.tensor(h.best_alpha), "act_scale": h.act_scale.detach().cpu(),
                      "scale": h.best_scale.detach().cpu(), "weight": m.weight.detach().cpu()}
    with torch.no_grad():
        res["out"] = model(data[0]).cpu()
    return res


def _case_sharded(dev, mtq, world_group: bool):
    from modelopt_amd.torch.quantization.sharded import (
        layer_shard_plan,
        layer_sharded_calibration,
        sync_sharded_amax,
    )

    g = torch.Generator().manual_seed(13)
    batches = [torch.randint(0, 64, (4, 24), generator=g).to(dev) for _ in range(3)]
    ids = torch.randint(0, 64, (2, 24), generator=g).to(dev)
    cfg = {**mtq.MXFP4_DEFAULT_CFG, "algorithm": "max"}

    def loop(m):
        with torch.no_grad():
            for b in batches:
                m(b)

    model = _tiny_llama(4).to(dev)
    n = -1
    if world_group:
        plan = layer_shard_plan(4, 0, 1)
        with layer_sharded_calibration(model, plan):
            mtq.quantize(model, cfg, loop)
        n = sync_sharded_amax(model, device=dev)
    else:
        mtq.quantize(model, cfg, loop)
    with torch.no_grad():
        logits = model(ids).logits.cpu()
    return {"amax": _amax_state(model, mtq), "logits": logits, "packed": torch.tensor(n)}


def _spy_collectives(dist):
    """Record (collective, tensor device, backend) of every call into ``sink[0]`` (one list per
    case; installed once, so the wrappers never stack)."""
    sink = [None]

    def wrap(name, tensor_pos):
        orig = getattr(dist, name)

        def f(*a, **k):
            t = a[tensor_pos] if len(a) > tensor_pos else None
            if isinstance(t, list):
                t = t[0] if t and isinstance(t[0], torch.Tensor) else None
            if sink[0] is not None:
                sink[0].append((name, t.device.type if isinstance(t, torch.Tensor) else "object",
                                dist.get_backend(k.get("group"))))
            return orig(*a, **k)

        setattr(dist, name, f)

    wrap("all_reduce", 0)
    wrap("all_gather", 1)
    wrap("all_gather_object", 1)
    return sink


def _worker(port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        import modelopt_amd.torch.quantization as mtq
        from modelopt_amd.torch.quantization.nn.modules import quant_module as qm

        calls: dict[str, list] = {}
        sink = _spy_collectives(dist)
        out = {}
        cases = {
            "fp8": lambda: _case_fp8(dev, mtq),
            "awq_fp32": lambda: _case_awq(dev, mtq, (16, 32, 16, 16), torch.float32, 8, 8),
            "awq_bf16_b128": lambda: _case_awq(dev, mtq, (256, 512, 256), torch.bfloat16, 128, 64),
        }
        for name, fn in cases.items():
            sink[0] = calls[name] = []
            dp = fn()
            prev, qm._DEFAULT_DP_GROUP = qm._DEFAULT_DP_GROUP, -1
            try:
                sink[0] = calls[name + "_nodist"] = []
                single = fn()
            finally:
                qm._DEFAULT_DP_GROUP = prev
            out[name] = {"dp": dp, "single": single}
        sink[0] = calls["sharded"] = []
        sh = _case_sharded(dev, mtq, True)
        sink[0] = None
        prev, qm._DEFAULT_DP_GROUP = qm._DEFAULT_DP_GROUP, -1
        try:
            single = _case_sharded(dev, mtq, False)
        finally:
            qm._DEFAULT_DP_GROUP = prev
        out["sharded"] = {"dp": sh, "single": single}
        buf = io.BytesIO()
        torch.save(out, buf)
        q.put((buf.getvalue(), json.dumps(calls)))
    except Exception as e:  # report instead of hanging the parent
        import traceback

        q.put((None, traceback.format_exc() + repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def world1_results(gpu):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        blob, info = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert blob is not None, info
    assert p.exitcode == 0, p.exitcode
    return torch.load(io.BytesIO(blob), weights_only=True), json.loads(info)


def _assert_same(a, b, where):
    if isinstance(a, dict):
        assert set(a) == set(b) and len(a) > 0, where
        for k in a:
            _assert_same(a[k], b[k], f"{where}.{k}")
        return
    assert a.dtype == b.dtype and a.shape == b.shape, where
    assert torch.equal(a.view(-1).view(torch.uint8) if a.numel() else a, b.view(-1).view(torch.uint8) if b.numel() else b), where


def _device_calls(calls, name, op):
    return [c for c in calls if c[0] == op and c[2] == "nccl" and c[1] == "cuda"]


@pytest.mark.timeout(300)
def test_nccl_max_calibrate_packed_all_reduce_on_device(world1_results):
    res, calls = world1_results
    assert _device_calls(calls["fp8"], "fp8", "all_reduce"), calls["fp8"]
    assert not calls["fp8_nodist"], calls["fp8_nodist"]
    _assert_same(res["fp8"]["dp"], res["fp8"]["single"], "fp8")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case", ["awq_fp32", "awq_bf16_b128"])
def test_nccl_awq_lite_fixed_order_sum_on_device(world1_results, case):
    res, calls = world1_results
    assert _device_calls(calls[case], case, "all_gather"), calls[case]
    assert all(c[1] != "cpu" for c in calls[case]), calls[case]  # no host staging under nccl
    assert not calls[case + "_nodist"], calls[case + "_nodist"]
    _assert_same(res[case]["dp"], res[case]["single"], case)
    assert len([k for k in res[case]["dp"] if k != "out"]) >= 2


@pytest.mark.timeout(300)
def test_nccl_sharded_sync_on_device(world1_results):
    res, calls = world1_results
    c = calls["sharded"]
    assert any(x[0] == "all_gather_object" and x[2] == "nccl" for x in c), c
    assert _device_calls(c, "sharded", "all_reduce"), c
    dp, single = res["sharded"]["dp"], res["sharded"]["single"]
    assert int(dp["packed"]) >= len(single["amax"]) > 0
    _assert_same(dp["amax"], single["amax"], "sharded.amax")
    _assert_same(dp["logits"], single["logits"], "sharded.logits")


@pytest.mark.timeout(300)
def test_bench_under_torchrun_nproc1_uses_nccl(gpu):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(REPO / "bench.py"),
           "--gpus", "1", "--steps", "5", "--warmup", "2", "--tokens", "4096",
           "--no-suite", "--no-cpu", "--no-ptq"]
    env = {**os.environ, "PYTHONUNBUFFERED": "1"}
    env.pop("MTQ_AMD_DIST_BACKEND", None)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240, env=env,
                          cwd=str(REPO))
    assert proc.returncode == 0, proc.stderr[-4000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.lstrip().startswith("{")]
    assert len(lines) == 1, proc.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["steps"] == 5
    assert line["config"]["dist_backend"] == "nccl", line["config"]
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
