#!/usr/bin/env python3
"""C4: MXFP4 (W+A, block 32, E8M0 scales) PTQ of Llama-3-70B with decoder layers sharded over
the ranks of one node: every rank builds the model on the meta device and
materialises only the embedding, the rotary tables and its own stage of layers (+ norm/lm_head on
the last rank), runs the same forward_loop, and hands hidden states to the next stage over RCCL
point-to-point; the stages' amax state is exchanged with one packed all_reduce(MAX).

    python scripts/ptq_sharded.py [--layers 80] [--samples 512] [--seq 512] [--batch 16]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 scripts/ptq_sharded.py

``--mode dp`` instead keeps a full replica per rank and splits the samples (288 GB HBM holds the
141 GB bf16 70B model), for comparison.  Random bf16 weights, synthetic token ids (no network).
"""

from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
for p in (str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

LLAMA3_70B = dict(
    hidden_size=8192,
    intermediate_size=28672,
    num_hidden_layers=80,
    num_attention_heads=64,
    num_key_value_heads=8,
    vocab_size=128256,
    max_position_embeddings=8192,
    rope_theta=500000.0,
    rms_norm_eps=1e-5,
)


@torch.no_grad()
def _materialize(module: torch.nn.Module, device, gen: torch.Generator):
    module.to_empty(device=device)
    for name, p in module.named_parameters():
        if p.dim() >= 2:
            p.normal_(0.0, 0.02, generator=gen)
        elif name.endswith("bias"):
            p.zero_()
        else:
            p.fill_(1.0)


def build_sharded(layers: int, device, plan=None):
    """Meta-build Llama-3-70B dims; materialise embedding, rotary, the owned layers (all if plan
    is None) and, on the last stage, norm + lm_head."""
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(**{**LLAMA3_70B, "num_hidden_layers": layers})
    cfg._attn_implementation = "sdpa"
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device("meta"):
            model = LlamaForCausalLM(cfg)
    finally:
        torch.set_default_dtype(prev)
    gen = torch.Generator(device=device).manual_seed(1234)
    owned = range(layers) if plan is None else plan.owned
    last = plan is None or plan.rank == plan.world - 1
    _materialize(model.model.embed_tokens, device, gen)
    for i in owned:
        g = torch.Generator(device=device).manual_seed(1234 + i)  # same weights whatever the split
        _materialize(model.model.layers[i], device, g)
    if last:
        _materialize(model.model.norm, device, gen)
        _materialize(model.lm_head, device, gen)
    rot = model.model.rotary_emb
    with torch.device(device):
        model.model.rotary_emb = type(rot)(config=cfg)
    return model.eval()


def run(samples=512, seq=512, batch=16, layers=80, config="MXFP4_DEFAULT_CFG", mode="pipeline",
        algorithm="max", eval_batches=4, baseline=True):
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.sharded import (
        layer_shard_plan,
        layer_sharded_calibration,
        sync_sharded_amax,
    )

    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    dev = torch.device("cuda", torch.cuda.current_device())
    plan = layer_shard_plan(layers, rank, world) if mode == "pipeline" else None
    t0 = time.perf_counter()
    model = build_sharded(layers, dev, plan)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    g = torch.Generator(device=dev).manual_seed(1234)
    ids = torch.randint(0, LLAMA3_70B["vocab_size"], (samples, seq), device=dev, generator=g)
    if mode == "dp":
        per = samples // world
        ids = ids[rank * per : (rank + 1) * per]
    batches = list(ids.split(batch))

    def forward_loop(m):
        with torch.no_grad():
            for b in batches:
                m(b)

    def ctx():
        return layer_sharded_calibration(model, plan) if mode == "pipeline" else contextlib.nullcontext()

    bf16_s = None
    if baseline:
        # the same forward passes without quantizers (the model's own bf16 cost of calibration)
        with ctx(), torch.no_grad():
            model(batches[0])
        torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()
        t0 = time.perf_counter()
        with ctx():
            forward_loop(model)
        torch.cuda.synchronize()
        bf16_s = _max_over_ranks(time.perf_counter() - t0, dev)

    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # MX presets are dynamic (algorithm None); "max" collects the per-tensor amax anyway so the
    # exported state carries it -- that is the amax the stages exchange
    cfg = {**getattr(mtq, config), "algorithm": None if algorithm == "none" else algorithm}

    with ctx():
        mtq.quantize(model, cfg, forward_loop)
    n_amax = sync_sharded_amax(model, device=dev) if mode == "pipeline" else None
    torch.cuda.synchronize()
    wall = _max_over_ranks(time.perf_counter() - t0, dev)

    # the fake-quant hot path at scale: MXFP4 W+A quantized forward over `eval_batches` batches
    ev = batches[:eval_batches]
    with ctx(), torch.no_grad():
        model(ev[0])  # warm-up
        torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()
        t0 = time.perf_counter()
        for b in ev:
            model(b)
        torch.cuda.synchronize()
    qfwd = _max_over_ranks(time.perf_counter() - t0, dev)
    res = {
        "model": f"Llama-3-70B dims, {layers} layers, bf16 random init", "config": config, "mode": mode,
        "world": world, "samples": samples, "seq": seq, "batch": batch,
        "stage_layers": None if plan is None else [plan.first, plan.last],
        "algorithm": algorithm,
        "ptq_wall_clock_s": round(wall, 3), "calib_tokens_per_s": round(samples * seq / wall, 1),
        "bf16_forward_loop_s": None if bf16_s is None else round(bf16_s, 3),
        "quantizer_overhead": None if bf16_s is None else round(wall / bf16_s - 1, 4),
        "qdq_forward_tokens_per_s": round(len(ev) * batch * seq * (1 if mode == "pipeline" else world) / qfwd, 1),
        "build_s": round(build_s, 1), "packed_amax_entries": n_amax,
        "hbm_gb_rank0": round(torch.cuda.max_memory_allocated() / 1e9, 1),
    }
    return res


def _max_over_ranks(v: float, dev) -> float:
    if dist.is_initialized():
        t = torch.tensor([v], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        v = float(t.item())
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=80)
    ap.add_argument("--samples", type=int, default=512)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--config", default="MXFP4_DEFAULT_CFG")
    ap.add_argument("--mode", choices=["pipeline", "dp"], default="pipeline")
    ap.add_argument("--algorithm", default="max", help='"max" or "none" (the MX preset as is)')
    ap.add_argument("--eval-batches", type=int, default=4)
    ap.add_argument("--no-baseline", action="store_true")
    ap.add_argument("--one-gpu", action="store_true",
                    help="all ranks on cuda:0 (a rehearsal of the N-rank pipeline on a one-GPU box)")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) or gloo (ranks sharing one GPU)")
    a = ap.parse_args()
    if "RANK" in os.environ:
        local = 0 if a.one_gpu else int(os.environ.get("LOCAL_RANK", 0))
        torch.cuda.set_device(local)
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(a.backend)
    else:
        torch.cuda.set_device(0)
    res = run(a.samples, a.seq, a.batch, a.layers, a.config, a.mode, a.algorithm, a.eval_batches,
              baseline=not a.no_baseline)
    res["backend"] = dist.get_backend() if dist.is_initialized() else None
    if not dist.is_initialized() or dist.get_rank() == 0:
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
