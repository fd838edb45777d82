#!/usr/bin/env python3
"""bench.py -- MI355X fake-quant throughput (G-elem/s, % of HBM roofline) + PTQ wall-clock.

Metric (BASELINE.json): "fake-quant G-elem/s (% HBM roofline) + PTQ wall-clock, Llama-3-8B FP8".

A *step* is one fake-quant pass of the hot path over one batch of synthetic Llama-shaped
activations resident in HBM: x bf16 [32768 tokens, 4096 hidden] (64 calibration samples x 512
tokens of Llama-3-8B's hidden size) through FP8 e4m3 static block-128 quant-dequant with a
precomputed per-block amax (the primary roofline target).  Inputs rotate over 4
buffers (1 GiB) so the 256 MiB Infinity Cache cannot serve them.  `value` = elements processed by
all ranks / slowest rank's time.

Also reported (same JSON line):
  roofline      dominant kernel: algorithmic bytes per launch / mean launch time (HIP events on
                the launch stream) vs 8.0 TB/s; `traffic` from the PMC profile in profiles/ if present
  kernels       per-kernel G-elem/s and % roofline for the other hot-path formats
  attention_p_qdq  the fused flash attention with softmax-P qdq, MFMA TFLOP/s per P mode
  awq_search    the AWQ-lite alpha search of one calibration batch on q_proj / gate_proj shapes:
                fused MFMA search call vs the batched hipBLASLt path it replaces (TFLOP/s, % peak)
  cpu_baseline  the oracle's restatement of the reference eager path (tensor_quant.py:46-59) timed
                on this host's cores on a bounded sample (rank 0, N=1 only)
  ptq           Llama-3-8B FP8 PTQ wall-clock (512 synthetic samples x 512 tokens; DP over ranks,
                slowest rank), the bf16 forward of the same batches at N=1, and the difference
  ptq_c3        Llama-3-8B INT4 AWQ-lite (block 128) PTQ wall-clock, same calibration set
  ptq_c5        Mixtral-8x7B FP8 PTQ wall-clock beside its bf16 forward (N=1 by default)
  ptq_c4        Llama-3-70B MXFP4 W+A PTQ wall-clock beside its bf16 forward: the whole model on one
                GPU at N=1, the decoder layers sharded over the ranks at N>1 (RCCL point-to-point
                hand-off between stages + one packed all_reduce(MAX) of the amax state)

Launch: python bench.py [--gpus N --steps K --warmup W].  N > 1 runs one rank per GPU: under
torch.distributed.run when RANK is set, otherwise bench.py starts that launcher itself as a child
process (before touching the GPU) and relays rank 0's JSON line and the exit status.
"""

from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "tensorrt-model-optimizer_amd"))
sys.path.insert(0, str(REPO))

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
TOKENS, HIDDEN, BLOCK = 32768, 4096, 128
N_BUF = 4


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(n_gpus: int) -> int:
    """`bench.py --gpus N` run directly (no RANK in the environment): start N ranks through a
    child `torch.distributed.run` (one process per GPU, rendezvous on 127.0.0.1), relay rank 0's
    stdout (the one JSON line) and return the launcher's exit status.  Nothing here touches the
    GPU, and the parent is not replaced (no exec): the ranks are its children.  Reference
    pattern: tests/_test_utils/torch/distributed/utils.py:56-67 (spawn_multiprocess_job)."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n_gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()),
           *sys.argv[1:]]
    print("bench: launching " + " ".join(cmd[1:]), file=sys.stderr, flush=True)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, env=os.environ.copy())
    lines = [ln for ln in proc.stdout.splitlines() if ln.strip()]
    for ln in lines:
        if ln.lstrip().startswith("{"):
            print(ln, flush=True)
        else:
            print(ln, file=sys.stderr, flush=True)
    if proc.returncode != 0:
        print(f"bench: a rank failed (launcher exit status {proc.returncode})", file=sys.stderr, flush=True)
    return proc.returncode


def _dist_init(n_gpus: int, device: str):
    cuda = device == "cuda"
    if n_gpus > 1 or "RANK" in os.environ:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        local = int(os.environ.get("LOCAL_RANK", 0))
        # MTQ_AMD_DIST_BACKEND=gloo rehearses the N>1 path with several ranks on one GPU (or on
        # the host kernels with --device cpu)
        backend = os.environ.get("MTQ_AMD_DIST_BACKEND", "nccl" if cuda else "gloo")
        if cuda:
            dev = local % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        return dist, dist.get_rank(), dist.get_world_size()
    if cuda:
        torch.cuda.set_device(0)
    return None, 0, 1


def _barrier(dist):
    if dist is not None:
        dist.barrier()


def _max_over_ranks(dist, v: float) -> float:
    if dist is None:
        return v
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([v], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_inputs(seed: int, device: str = "cuda", tokens: int = TOKENS):
    g = torch.Generator(device=device).manual_seed(seed)
    xs = []
    for i in range(N_BUF):
        x = torch.randn(tokens, HIDDEN, device=device, dtype=torch.bfloat16, generator=g)
        # 0.1 % outlier columns x16
        cols = torch.randperm(HIDDEN, device=device, generator=g)[: HIDDEN // 1000]
        x[:, cols] *= 16
        xs.append(x)
    return xs


def time_kernel(fn, xs, steps: int, warmup: int, dist=None):
    """Run fn over rotating inputs; returns (wall seconds for `steps`, mean ms per launch).

    The mean launch duration comes from one pair of HIP events recorded on the launch stream
    around the whole timed region, divided by `steps` (back-to-back launches, so inter-kernel
    gaps count against it).  Events around every single launch would add their own GPU-side
    packets to each step (measured: ~4 us per launch on a ~87 us kernel).  Host tensors (the
    --device cpu rehearsal) are timed by the wall clock alone."""
    outs = [None] * len(xs)
    for i in range(warmup):
        outs[i % len(xs)] = fn(xs[i % len(xs)])
    if not xs[0].is_cuda:
        _barrier(dist)
        t0 = time.perf_counter()
        for i in range(steps):
            outs[i % len(xs)] = fn(xs[i % len(xs)])
        _barrier(dist)
        wall = time.perf_counter() - t0
        return wall, wall * 1e3 / steps
    torch.cuda.synchronize()
    _barrier(dist)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for i in range(steps):
        outs[i % len(xs)] = fn(xs[i % len(xs)])
    e1.record(stream)
    torch.cuda.synchronize()
    _barrier(dist)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / steps
    return wall, ms


def kernel_suite(ops, xs, steps, warmup):
    """Secondary per-kernel numbers (one rank)."""
    n = xs[0].numel()
    res = {}
    amax_t = torch.tensor(8.0, device="cuda")
    blk = [x.view(-1, BLOCK).abs().amax(dim=1, keepdim=True).float() for x in xs]
    rows = [x.abs().amax(dim=1, keepdim=True).float() for x in xs]
    rows_own = [r.to(x.dtype) for r, x in zip(rows, xs)]  # what mtq stores for a bf16 model's weights
    cases = {
        "fp8_per_tensor": (lambda x: ops.fake_e4m3fy(x, amax_t), 4),
        "int8_per_tensor": (lambda x: ops.fake_tensor_quant(x, amax_t, 8, False, False), 4),
        "int8_per_channel_axis0": (
            lambda x: ops.quantize_op(x, rows[[id(t) for t in xs].index(id(x))], 8, 0, False, False), 4),
        "int8_per_channel_axis0_bf16amax": (
            lambda x: ops.quantize_op(x, rows_own[[id(t) for t in xs].index(id(x))], 8, 0, False, False), 4),
        "int4_block128_static": (
            lambda x: ops.quantize_op(x.view(-1, BLOCK), blk[[id(t) for t in xs].index(id(x))], 4, 0, False, False), 4),
        "mxfp4_block32_dynamic": (lambda x: ops.fused_amax_convert(x, 32, 6, 9, None), 4),
        "mxfp8_block32_dynamic": (lambda x: ops.fused_amax_convert(x, 32, 0, 9, None), 4),
        "int4_block128_dynamic_awq": (lambda x: ops.block_quant_dynamic(x, None, 128, 4, False, False), 4),
        "nvfp4_block16_dynamic": (lambda x: ops.nvfp4_fake_quant_block(x, amax_t, 16), 4),
        # checkpoint export packing: bf16 read + packed bytes written
        "export_fp8_per_tensor": (lambda x: ops.export_fp8(x, fp8_s, False, True), 3),
        # (bytes per element: bf16 in + packed codes out + the block scales read / written --
        # NVFP4 fp32 per 16, INT4 fp32 per 128, MXFP4 E8M0 bytes per 32 -- each input with its own
        # scale tensor, as every weight of a real export has)
        "export_nvfp4_pack": (lambda x: ops.export_nvfp4(x, nv_bs[ix(x)], nv_s2), 2.5 + 4 / 16),
        "export_int4_pack": (lambda x: ops.export_int4(x, i4_s[ix(x)]), 2.5 + 4 / 128),
        "export_mxfp4_pack": (lambda x: ops.export_mxfp4(x, 32)[0], 2.5 + 1 / 32),
        "export_fp8_block2d_128": (lambda x: ops.export_fp8_block2d(x, b2d_s[ix(x)], 128, 128), 3 + 4 / 16384),
        "amax_per_tensor": (None, 2),
        # K6 per-row (axis 0 kept) and per-column (axis -1 kept) running amax, K7 histogram
        "amax_per_row": (lambda x: ops.amax_accumulate(x, acc_r, 1, x.shape[0], x.shape[1]) or acc_r, 2),
        "amax_per_column": (lambda x: ops.amax_accumulate(x, acc_c, x.shape[0], x.shape[1], 1) or acc_c, 2),
        "histogram_2048_abs": (lambda x: ops.histogram_abs_accumulate(x, hmax, counts, 2048, False) or counts, 2),
    }
    acc_r = torch.zeros(xs[0].shape[0], device="cuda")
    acc_c = torch.zeros(xs[0].shape[1], device="cuda")
    hmax = torch.tensor([16.0 * 6], device="cuda")
    counts = torch.zeros(2048, dtype=torch.int32, device="cuda")
    ids = [id(t) for t in xs]

    def ix(x):
        return ids.index(id(x))

    nv_bs = [torch.ones(x.numel() // 16, device="cuda") for x in xs]
    # the packers' scale inputs, computed once (a per-call division would time a second launch).
    # FP8 export: the scale an export derives from the tensor itself, amax / 448 (quant_utils.py
    # per-tensor weight scale; one scale over the 4 rotating inputs), so no quotient passes 448 --
    # with the fake-quant legs' amax 8, the x16 outlier columns overflowed in ~0.5 % of the lanes
    # and a quarter of the waves ran the exact out-of-range path (0.72 vs 0.78-0.79, r05k)
    fp8_s = torch.stack([x.abs().amax().float() for x in xs]).amax() / 448
    nv_s2 = amax_t / 2688
    i4_s = [torch.full((x.shape[0], x.shape[1] // 128), 0.01, device="cuda") for x in xs]
    # FP8_PB_WO export: each input's own 128 x 128 block amax / 448 (fp32), as the export derives it
    b2d_s = [x.view(x.shape[0] // 128, 128, x.shape[1] // 128, 128).abs().amax(dim=(1, 3)).float() / 448 for x in xs]
    acc = torch.zeros(1, device="cuda")
    for name, (fn, bpe) in cases.items():
        if fn is None:
            def fn(x):  # noqa: E306
                ops.amax_accumulate(x, acc, 1, 1, x.numel())
                return acc
        _, ms = time_kernel(fn, xs, max(steps, 10), warmup)
        gbs = n * bpe / (ms * 1e-3) / 1e9
        res[name] = {
            "gelem_s": round(n / (ms * 1e-3) / 1e9, 1),
            "GB_s": round(gbs, 1),
            "frac": round(gbs / HBM_PEAK_GBS, 4),
            "ms": round(ms, 4),
        }
    # the calibrator's >2^24-element call ([8192, 14336] = 117.4 M elements, an MLP down_proj
    # input): torch.histc's per-thread fp32 chunks (16 = the box's CPU share), each counted exactly
    # and clamped at 2^24, beside one exact-count launch over the same tensor
    from modelopt_amd.torch.quantization.calib.histogram import _histc_counts  # noqa: PLC0415

    big = [torch.randn(8192, 14336, device="cuda", generator=torch.Generator(device="cuda").manual_seed(7))
           .to(torch.bfloat16)]
    nb = big[0].numel()
    for name, fn in {
        "histogram_2048_abs_117M_histc16": lambda x: _histc_counts(x, hmax, 2048, False, threads=16),
        "histogram_2048_abs_117M_histc16_skip_zeros": lambda x: _histc_counts(x, hmax, 2048, True, threads=16),
        "histogram_2048_abs_117M_exact": lambda x: ops.histogram_abs_accumulate(x, hmax, counts, 2048, False) or counts,
    }.items():
        _, ms = time_kernel(fn, big, max(steps // 2, 5), min(warmup, 3))
        gbs = nb * 2 / (ms * 1e-3) / 1e9
        res[name] = {"gelem_s": round(nb / (ms * 1e-3) / 1e9, 1), "GB_s": round(gbs, 1),
                     "frac": round(gbs / HBM_PEAK_GBS, 4), "ms": round(ms, 4), "elements": nb}
    del big
    return res


def attention_suite(iters: int = 50):
    """The fused flash attention with softmax-P qdq (mtq_attention_fwd) on a Llama-3-8B
    calibration batch (16 x 512 tokens, 32 / 8 heads, D 128, bf16, causal): MFMA TFLOP/s per P
    mode vs the 2.5 PF dense bf16 peak, beside torch SDPA without P qdq."""
    from benchmarks import attention as bench_attention  # noqa: PLC0415

    r = bench_attention.measure(iters=iters)
    peak = r["peak_tflops_bf16_dense"]
    for v in list(r["modes"].values()) + [r["sdpa_no_qdq"], r["eager_fp8_p"]]:
        v["frac_mfma_peak"] = round(v["tflops"] / peak, 4)
    return r


def awq_search_suite(rounds: int = 3):
    """N1: the AWQ-lite alpha search of one calibration batch (8192 tokens, 11 alphas) on
    Llama-3-8B's q_proj and gate_proj shapes -- the fused call (x * (1/s) pass + the W4 MFMA
    search kernel with the loss in its epilogue, mtq_awq_search_gemm) beside the batched path it
    replaces (the same pass + 11 hipBLASLt GEMMs + one loss pass) and the 11 GEMMs alone; MFMA
    TFLOP/s = 2 M N K G / time against the 2.5 PF dense bf16 peak.  Interleaved rounds, medians."""
    import statistics  # noqa: PLC0415

    import torch.nn.functional as F  # noqa: PLC0415

    from modelopt_amd import _ext  # noqa: PLC0415

    ops = _ext.ops()
    M, G, res = 8192, 11, {}
    for name, (N, K) in {"q_proj": (4096, 4096), "gate_proj": (14336, 4096)}.items():
        gen = torch.Generator(device="cuda").manual_seed(N + K)
        x = torch.randn(M, K, device="cuda", generator=gen).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda", generator=gen) * 0.02).to(torch.bfloat16)
        s = torch.rand(G, K, device="cuda", generator=gen) * 3 + 0.25
        si = (1 / s).to(torch.bfloat16)
        wq = ops.block_quant_dynamic_multi(w, s.to(torch.bfloat16), 128, 4, False, False)
        yref = F.linear(x, w)
        loss = torch.zeros(G, device="cuda")
        out = torch.empty((G, M, N), dtype=x.dtype, device="cuda")

        def fused():
            ops.awq_search_gemm(x, si, wq, None, yref, loss)

        def batched():
            xs = ops.awq_prescale(x, si)
            for g in range(G):
                torch.mm(xs[g], wq[g].t(), out=out[g])
            ops.awq_mse_multi(out, yref, loss)

        def gemms():
            for g in range(G):
                torch.mm(x, wq[g].t(), out=out[g])

        arms = {"fused_search": fused, "batched_hipblaslt_path": batched, "hipblaslt_gemms_alone": gemms}
        t = {k: [] for k in arms}
        names = list(arms)
        for r_ in range(rounds):  # the order rotates per round (a fixed order biases an arm by ~4 %)
            for k in names[r_ % len(names):] + names[:r_ % len(names)]:
                f = arms[k]
                f()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    f()
                e1.record()
                torch.cuda.synchronize()
                t[k].append(e0.elapsed_time(e1) / 3)
        flop = 2.0 * M * N * K * G
        r = {k: {"ms": round(statistics.median(v), 3),
                 "tflops": round(flop / (statistics.median(v) * 1e-3) / 1e12, 1)} for k, v in t.items()}
        for v in r.values():
            v["frac_mfma_peak"] = round(v["tflops"] / 2500.0, 4)
        r["fused_speedup_vs_batched"] = round(r["batched_hipblaslt_path"]["ms"] / r["fused_search"]["ms"], 3)
        res[name] = r
        del x, w, wq, yref, out
    torch.cuda.empty_cache()
    return {"tokens": M, "alphas": G, "dtype": "bf16", "shapes": res}


def host_cpu_info():
    """Physical cores of the host (unique (package, core) pairs in /proc/cpuinfo), the CPUs this
    process may run on, and torch's intra-op thread count."""
    phys = set()
    try:
        pkg = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k = k.strip()
            if k == "physical id":
                pkg = v.strip()
            elif k == "core id":
                core = v.strip()
            elif not k and pkg is not None:
                phys.add((pkg, core))
                pkg = core = None
        if pkg is not None:
            phys.add((pkg, core))
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count()
    return {"host_physical_cores": len(phys) or None, "process_cpus": allowed,
            "torch_threads": torch.get_num_threads()}


def _time_fp8_eager(R, xb, amax, target_s):
    R.fp8_eager(xb, amax)  # warm-up
    passes, t0 = 0, time.perf_counter()
    while True:
        R.fp8_eager(xb, amax)
        passes += 1
        el = time.perf_counter() - t0
        if el >= target_s or passes >= 200:
            return passes, el


def cpu_baseline(target_s: float = 10.0):
    """Oracle restatement of the reference eager FP8 block path, timed on host cores: all the
    threads torch uses here (the box's per-job CPU share) and one thread."""
    from oracle import ref_ops as R  # test infrastructure: the checker / CPU baseline only

    rows = 8192  # bounded sample: [8192, 4096] bf16 = 33.5 M elements per pass
    g = torch.Generator().manual_seed(1234)
    x = torch.randn(rows, HIDDEN, generator=g).to(torch.bfloat16)
    xb = x.view(-1, BLOCK)
    amax = xb.abs().amax(dim=1, keepdim=True).float()
    info = host_cpu_info()
    passes, el = _time_fp8_eager(R, xb, amax, target_s)
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:  # the same sample (a smaller one would sit in the host caches and read faster)
        xs1 = xb
        p1, el1 = _time_fp8_eager(R, xs1, amax, target_s / 2)
    finally:
        torch.set_num_threads(nt)
    return {
        "value": round(passes * x.numel() / el / 1e9, 4),
        "unit": "G-elem/s",
        "cores": nt,
        "kind": "port",
        "sample": f"{passes} passes of FP8 e4m3 static block-128 fake-quant (oracle fp8_eager, the "
        f"reference _fp8_eager ATen sequence) over bf16 [{rows}, {HIDDEN}], {el:.1f} s, {nt} threads",
        "cores_basis": (
            f"torch intra-op threads = {nt} (OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}): "
            f"the job's CPU share on the shared GPU box, not the host's {info['host_physical_cores']} "
            f"physical cores ({info['process_cpus']} CPUs in the affinity mask are shared with other jobs)"
        ),
        "one_thread": {
            "value": round(p1 * xs1.numel() / el1 / 1e9, 4),
            "unit": "G-elem/s",
            "cores": 1,
            "sample": f"{p1} passes over bf16 [{rows}, {HIDDEN}], {el1:.1f} s",
        },
        **info,
    }


def cpu_e2e_baseline(samples: int = 8):
    """SURVEY §8d E2E CPU baseline: one Llama-3-8B decoder layer (bf16, random init), max
    calibration of its 7 linears (input amax per batch + weight amax, the oracle's reduce_amax =
    the reference ATen sequence) over `samples` x 512 tokens on the host cores; reported per layer
    per sample, with the full 32-layer x 512-sample extrapolation labelled as such."""
    from transformers import LlamaConfig
    from transformers.models.llama.modeling_llama import LlamaDecoderLayer, LlamaRotaryEmbedding

    from oracle import ref_ops as R  # test infrastructure: the CPU baseline only

    from benchmarks.ptq_llama import LLAMA3_8B

    cfg = LlamaConfig(**LLAMA3_8B)
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(1234)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        layer = LlamaDecoderLayer(cfg, 0).eval()
        rope = LlamaRotaryEmbedding(cfg)
    finally:
        torch.set_default_dtype(prev)
    amax = {}

    def hook(mod, args):
        a = R.reduce_amax(args[0], axis=None)
        amax[mod] = a if mod not in amax else torch.maximum(amax[mod], a)
        if ("w", mod) not in amax:
            amax[("w", mod)] = R.reduce_amax(mod.weight, axis=None)

    hs = [m.register_forward_pre_hook(hook) for m in layer.modules() if isinstance(m, torch.nn.Linear)]
    g = torch.Generator().manual_seed(1234)
    x = (torch.randn(samples, 512, cfg.hidden_size, generator=g) * 0.5).to(torch.bfloat16)
    pos = torch.arange(512)[None].expand(samples, -1)
    t0 = time.perf_counter()
    with torch.no_grad():
        pe = rope(x, pos)
        for i in range(0, samples, 4):
            layer(x[i : i + 4], position_embeddings=(pe[0][i : i + 4], pe[1][i : i + 4]), attention_mask=None)
    el = time.perf_counter() - t0
    for h in hs:
        h.remove()
    per = el / samples
    return {
        "value": round(per, 4),
        "unit": "s per decoder layer per 512-token sample",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "sample": f"Llama-3-8B decoder layer, bf16, {samples} x 512 tokens, max calibration of 7 linears "
        f"(oracle reduce_amax), {el:.1f} s",
        "extrapolated_ptq_wall_clock_s": round(per * 32 * 512, 1),
        "extrapolation": "per-layer-per-sample x 32 layers x 512 samples (labelled estimate, not run)",
    }


def load_traffic():
    """HBM bytes per launch of the dominant kernel from the committed PMC profile, if any."""
    for p in sorted((REPO / "profiles").glob("traffic_*.json"), reverse=True):
        try:
            d = json.loads(p.read_text())
            if d.get("kernel_config") == f"fp8_block{BLOCK}_bf16_{TOKENS}x{HIDDEN}":
                return d.get("hbm_bytes_per_launch"), p.name
        except Exception:  # noqa: BLE001
            continue
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-suite", action="store_true", help="skip the secondary kernel table")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-ptq", action="store_true", help="skip the Llama-3-8B FP8 PTQ wall-clock")
    ap.add_argument("--no-c3", action="store_true", help="skip the Llama-3-8B INT4 AWQ-lite PTQ (C3)")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip C5: Mixtral-8x7B FP8 PTQ (93 GB bf16 resident, ~40 s) beside its bf16 forward; it runs "
                    "by default at N=1")
    ap.add_argument("--c5", action="store_true", help="run C5 at N > 1 too (data-parallel, 93 GB per rank)")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip C4: Llama-3-70B MXFP4 W+A PTQ (141 GB bf16 at N=1; layer-sharded over the ranks at N>1)")
    ap.add_argument("--c4-dims", choices=("llama3-70b", "tiny"), default=None,
                    help="C4 model dims (default: llama3-70b on the GPU, tiny for the --device cpu rehearsal)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--device", choices=("cuda", "cpu"), default=None,
                    help="cpu = plumbing rehearsal on the product's host kernels (default: cuda when a "
                    "GPU is visible, else cpu)")
    ap.add_argument("--tokens", type=int, default=TOKENS, help="rows per rank (default: the K3 workload)")
    args = ap.parse_args()

    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(_self_launch(args.gpus))
    device = args.device or ("cuda" if torch.cuda.is_available() else "cpu")
    # the GPU-only legs need a device; the C4 leg's plumbing (layer-sharded pipeline, packed
    # amax exchange) also runs on the host at tiny dims
    run_c4 = not (args.no_ptq or args.no_c4)
    if device == "cpu":
        args.no_suite = args.no_ptq = True
    dist, rank, world = _dist_init(args.gpus, device)
    from modelopt_amd import _ext

    ops = _ext.ops()
    tokens = args.tokens
    xs = make_inputs(1234 + rank, device, tokens)
    blk = [x.view(-1, BLOCK).abs().amax(dim=1, keepdim=True).float() for x in xs]
    idx = {id(x): i for i, x in enumerate(xs)}

    def step(x):
        return ops.quantize_op(x.view(-1, BLOCK), blk[idx[id(x)]], 8, 4, False, False)

    wall, ms = time_kernel(step, xs, args.steps, args.warmup, dist)
    wall = _max_over_ranks(dist, wall)
    n = xs[0].numel()
    total = n * args.steps * world
    value = total / wall / 1e9
    alg_bytes = n * 4 + (n // BLOCK) * 4  # read x bf16 + write y bf16 + read fp32 amax
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic() if (device == "cuda" and tokens == TOKENS) else (None, None)

    out = {
        "metric": "fake-quant G-elem/s (% HBM roofline) + PTQ wall-clock, Llama-3-8B FP8",
        "value": round(value, 2),
        "unit": "G-elem/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (seeded randn bf16, 0.1% outlier columns x16; amax precomputed per block)",
        "config": {
            "workload": "FP8 e4m3 static block-128 fake quant-dequant of Llama-3-8B activations "
            f"[{tokens} tokens x {HIDDEN}] bf16 per rank (SURVEY K3)",
            "tokens_per_rank": tokens,
            "hidden": HIDDEN,
            "block": BLOCK,
            "parallelism": f"dp{world}",
            "sharding": "independent row shards per rank, no collective in the timed path",
            "dist_backend": dist.get_backend() if dist is not None else None,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": "ew_group_sk_kernel<bf16, Fp8AxisVecOp, U=2, LPB=8> (scalar-loaded block amax) via modelopt_amd::quantize_op",
            "algorithmic_bytes_per_launch": alg_bytes,
            "mean_launch_ms": round(ms, 4),
        },
    }
    if device == "cpu":
        out["device"] = "cpu (plumbing rehearsal on the product's host kernels: not an MI355X measurement)"
        out["roofline"]["kernel"] = "mtq_cpu_fake_e4m3fy (host)"
    if rank == 0 and not args.no_suite:
        out["kernels"] = kernel_suite(ops, xs, args.steps, args.warmup)
        out["attention_p_qdq"] = attention_suite()
        out["awq_search"] = awq_search_suite()
    if not args.no_ptq:
        from benchmarks import ptq_llama  # noqa: PLC0415

        del xs, blk
        torch.cuda.empty_cache()
        _barrier(dist)
        # the library's conversion messages (reference prints) go to stderr: stdout carries
        # exactly one JSON line
        with contextlib.redirect_stdout(sys.stderr):
            res = ptq_llama.run(samples=512, seq=512, rank=rank, world=world, baseline=(world == 1))
        res["ptq_wall_clock_s"] = round(_max_over_ranks(dist, res["ptq_wall_clock_s"]), 3)
        res["calib_tokens_per_s"] = round(512 * 512 / res["ptq_wall_clock_s"], 1)
        out["ptq"] = res
        if not args.no_c3:
            # C3: INT4 AWQ-lite (block 128) on the same model and calibration set
            print("bench: C3 INT4_AWQ_CFG PTQ ...", file=sys.stderr, flush=True)
            _barrier(dist)
            with contextlib.redirect_stdout(sys.stderr):
                r3 = ptq_llama.run(samples=512, seq=512, rank=rank, world=world, baseline=False,
                                   config="INT4_AWQ_CFG")
            r3["ptq_wall_clock_s"] = round(_max_over_ranks(dist, r3["ptq_wall_clock_s"]), 3)
            r3["calib_tokens_per_s"] = round(512 * 512 / r3["ptq_wall_clock_s"], 1)
            out["ptq_c3"] = r3
        if not args.no_c5 and (world == 1 or args.c5):
            # C5: Mixtral-8x7B FP8 PTQ over the MoE QuantLinear path (a 93 GB model per rank)
            print("bench: C5 Mixtral-8x7B FP8_DEFAULT_CFG PTQ ...", file=sys.stderr, flush=True)
            torch.cuda.empty_cache()
            _barrier(dist)
            with contextlib.redirect_stdout(sys.stderr):
                r5 = ptq_llama.run(samples=512, seq=512, rank=rank, world=world, baseline=(world == 1),
                                   model_name="mixtral-8x7b")
            r5["ptq_wall_clock_s"] = round(_max_over_ranks(dist, r5["ptq_wall_clock_s"]), 3)
            r5["calib_tokens_per_s"] = round(512 * 512 / r5["ptq_wall_clock_s"], 1)
            if "bf16_forward_s" in r5:
                r5["overhead_frac"] = round(r5["ptq_wall_clock_s"] / r5["bf16_forward_s"] - 1.0, 4)
            out["ptq_c5"] = r5
    if run_c4:
        # C4: Llama-3-70B MXFP4 W+A (block 32, E8M0) PTQ; whole model at N=1, layer-sharded at N>1
        from benchmarks import ptq_c4  # noqa: PLC0415

        dims = args.c4_dims or ("tiny" if device == "cpu" else "llama3-70b")
        print(f"bench: C4 {dims} MXFP4_DEFAULT_CFG PTQ ...", file=sys.stderr, flush=True)
        if device == "cuda":
            torch.cuda.empty_cache()
        _barrier(dist)
        small = dict(samples=16, seq=64, batch=4) if dims == "tiny" else dict(samples=512, seq=512, batch=16)
        with contextlib.redirect_stdout(sys.stderr):
            out["ptq_c4"] = ptq_c4.run(**small, dims=dims, baseline=True,
                                       device=torch.device("cuda", torch.cuda.current_device()) if device == "cuda"
                                       else torch.device("cpu"))
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        if not args.no_ptq:
            out["cpu_baseline"]["ptq_e2e"] = cpu_e2e_baseline()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
