#!/usr/bin/env python3
"""C4: MXFP4 (E2M1 elements, block 32, E8M0 scales) weight + activation PTQ of Llama-3-70B, with
the decoder layers sharded over the ranks of one node (BASELINE config C4).

* N = 1: the whole model on one GPU (141 GB bf16 fits in the 288 GB of HBM), plain
  ``mtq.quantize(model, MXFP4_DEFAULT_CFG + max, forward_loop)``.
* N > 1: every rank builds the model on the meta device and materialises the embedding, the
  rotary tables and only its own contiguous stage of decoder layers (+ norm / lm_head on the last
  rank; 80 layers / 8 GPUs = 10 per GPU); the unchanged ``forward_loop`` runs on every rank inside
  ``layer_sharded_calibration``, which hands the hidden states to the next stage with RCCL
  point-to-point (``isend`` / ``recv`` over xGMI, sharded.py), and ``sync_sharded_amax`` then gives
  every rank the whole quantizer state with ONE packed fp32 ``all_reduce(MAX)``.

The MX presets are dynamic (``algorithm`` None in the reference); ``"max"`` collects the
per-tensor amax anyway so the exported state carries it -- that is the amax the stages exchange.
Reference: model_calib.py:2051-2189 (layerwise calibration, the per-layer unit),
examples/hf_ptq/example_utils.py:758-880 (device-map layer placement), tensor_quantizer.py:1373-1385
(amax sync).  Random bf16 weights (per-layer seeds, so a layer's weights do not depend on the
split) and synthetic token ids: there is no network for checkpoints or datasets.

``device="cpu"`` with ``dims="tiny"`` rehearses the same plumbing on the host (gloo P2P and
all-reduce, the product's CPU amax kernel); the quantized evaluation forward is skipped there
because the MX qdq op has no CPU kernel.

    python benchmarks/ptq_c4.py [--layers 80] [--samples 512] [--seq 512] [--batch 16]
"""

from __future__ import annotations

import argparse
import contextlib
import gc
import json
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
# host rehearsal: the same architecture at toy width (every dimension a multiple of the MX block)
TINY = dict(
    hidden_size=64,
    intermediate_size=128,
    num_hidden_layers=4,
    num_attention_heads=4,
    num_key_value_heads=2,
    vocab_size=256,
    max_position_embeddings=512,
    rope_theta=500000.0,
    rms_norm_eps=1e-5,
)
DIMS = {"llama3-70b": ("Llama-3-70B", LLAMA3_70B), "tiny": ("tiny Llama", TINY)}


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


def build(dims: str, layers: int, device, plan=None):
    """Meta-build the model; materialise the embedding, the rotary tables, the owned decoder layers
    (all of them when ``plan`` is None) and, on the last stage, the final norm + lm_head."""
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(**{**DIMS[dims][1], "num_hidden_layers": layers})
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


def amax_digest(model):
    """(number of enabled quantizers holding a real amax, sha256 of their names + fp32 amax bytes
    in name order)."""
    import hashlib

    from modelopt_amd.torch.quantization.nn import TensorQuantizer

    h, n = hashlib.sha256(), 0
    for name, m in sorted(model.named_modules(), key=lambda kv: kv[0]):
        a = getattr(m, "_amax", None) if isinstance(m, TensorQuantizer) and m.is_enabled else None
        if isinstance(a, torch.Tensor) and a.device.type != "meta":
            n += 1
            h.update(name.encode())
            h.update(a.detach().float().cpu().contiguous().numpy().tobytes())
    return n, h.hexdigest()


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def _barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def _max_over_ranks(v: float, dev) -> float:
    if dist.is_available() and dist.is_initialized():
        on = dev if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([v], device=on, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        v = float(t.item())
    return v


def run(samples=512, seq=512, batch=16, layers=None, dims="llama3-70b", config="MXFP4_DEFAULT_CFG",
        algorithm="max", baseline=True, eval_batches=4, device=None):
    """One C4 PTQ; returns the JSON-able result (identical on every rank; max-over-ranks times)."""
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization.sharded import (
        layer_shard_plan,
        layer_sharded_calibration,
        sync_sharded_amax,
    )

    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    dev = torch.device(device)
    label, d = DIMS[dims]
    layers = layers or d["num_hidden_layers"]
    plan = layer_shard_plan(layers, rank, world) if world > 1 else None
    t0 = time.perf_counter()
    model = build(dims, layers, dev, plan)
    _sync(dev)
    build_s = time.perf_counter() - t0
    g = torch.Generator(device=dev).manual_seed(1234)
    ids = torch.randint(0, d["vocab_size"], (samples, seq), device=dev, generator=g)
    batches = list(ids.split(batch))

    def forward_loop(m):
        with torch.no_grad():
            for b in batches:
                m(b)

    def ctx():
        return layer_sharded_calibration(model, plan) if plan is not None else contextlib.nullcontext()

    res = {"model": f"{label} dims, {layers} layers, bf16 random init", "config": config,
           "algorithm": algorithm, "world": world, "samples": samples, "seq": seq, "batch": batch,
           "mode": "layer-sharded pipeline (P2P hand-off between stages + one packed all_reduce(MAX))" if plan is not None
           else "whole model on one device",
           "stage_layers": None if plan is None else [plan.first, plan.last],
           "dist_backend": dist.get_backend() if world > 1 else None,
           "build_s": round(build_s, 2)}
    if baseline:
        # the same forward passes without quantizers: the model's own bf16 cost of calibration
        with ctx(), torch.no_grad():
            model(batches[0])  # warm-up (kernels, allocator)
        gc.collect()
        _sync(dev)
        _barrier()
        t0 = time.perf_counter()
        with ctx():
            forward_loop(model)
        _sync(dev)
        res["bf16_forward_s"] = round(_max_over_ranks(time.perf_counter() - t0, dev), 3)

    cfg = {**getattr(mtq, config), "algorithm": None if algorithm == "none" else algorithm}
    gc.collect()
    _sync(dev)
    _barrier()
    t0 = time.perf_counter()
    with ctx():
        mtq.quantize(model, cfg, forward_loop)
    n_packed = sync_sharded_amax(model, device=dev) if plan is not None else None
    _sync(dev)
    res["ptq_wall_clock_s"] = round(_max_over_ranks(time.perf_counter() - t0, dev), 3)
    res["calib_tokens_per_s"] = round(samples * seq / res["ptq_wall_clock_s"], 1)
    if baseline:
        res["overhead_frac"] = round(res["ptq_wall_clock_s"] / res["bf16_forward_s"] - 1.0, 4)
    res["enabled_quantizers"] = sum(1 for _, m in model.named_modules()
                                    if isinstance(m, mtq.TensorQuantizer) and m.is_enabled)
    res["packed_amax_entries"] = n_packed
    # every quantizer holds its amax on every rank after the exchange (the non-owners' from it)
    n_amax, digest = amax_digest(model)
    res["quantizers_with_amax"] = n_amax
    # sha256 over every quantizer's (name, fp32 amax bytes): equal at every N when the layer-sharded
    # run reproduces the single-device calibration bit for bit
    res["amax_sha256"] = digest

    if dev.type == "cuda" and eval_batches:
        # the fake-quant hot path at scale: the MXFP4 W+A quantized forward
        ev = batches[:eval_batches]
        with ctx(), torch.no_grad():
            out = model(ev[0])  # warm-up
            _sync(dev)
            _barrier()
            t0 = time.perf_counter()
            for b in ev:
                out = model(b)
            _sync(dev)
        qfwd = _max_over_ranks(time.perf_counter() - t0, dev)
        res["qdq_forward_tokens_per_s"] = round(len(ev) * batch * seq / qfwd, 1)
        if out is not None:  # the last stage (or the whole model) holds the logits
            res["finite_logits"] = bool(torch.isfinite(out.logits).all())
    else:
        res["qdq_forward_tokens_per_s"] = None  # MX qdq has no host kernel
    if dev.type == "cuda":
        res["hbm_gb_peak_rank"] = round(_max_over_ranks(torch.cuda.max_memory_allocated(dev) / 1e9, dev), 1)
    del model
    gc.collect()
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    return res


def main():
    import os

    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", default="llama3-70b", choices=sorted(DIMS))
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--samples", type=int, default=512)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--config", default="MXFP4_DEFAULT_CFG")
    ap.add_argument("--algorithm", default="max", help='"max" or "none" (the MX preset as is)')
    ap.add_argument("--eval-batches", type=int, default=4)
    ap.add_argument("--no-baseline", action="store_true")
    ap.add_argument("--one-gpu", action="store_true",
                    help="all ranks on cuda:0 (a rehearsal of the N-rank pipeline on a one-GPU box)")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) or gloo (ranks sharing one GPU / the host)")
    a = ap.parse_args()
    dev = None
    if "RANK" in os.environ:
        if torch.cuda.is_available():
            local = 0 if a.one_gpu else int(os.environ.get("LOCAL_RANK", 0))
            torch.cuda.set_device(local)
            dev = torch.device("cuda", local)
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(0)
    res = run(a.samples, a.seq, a.batch, a.layers, a.dims, a.config, a.algorithm, not a.no_baseline,
              a.eval_batches, dev)
    if not dist.is_initialized() or dist.get_rank() == 0:
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
