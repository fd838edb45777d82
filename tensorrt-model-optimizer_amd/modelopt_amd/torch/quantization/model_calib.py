"""Calibration algorithms of the PTQ hot path (reference: model_calib.py).

* ``max_calibrate`` (reference :311-498): weight-only collect, ``forward_loop`` collect, load amax,
  then ONE packed ``all_reduce(MAX)`` of every quantizer's amax per call (the reference issues one
  collective per quantizer, :390-407 -> tensor_quantizer.py:1373).  MAX is exact and associative,
  so the packed exchange is bit-identical to the per-quantizer one for any world size.
* ``awq_lite`` (reference :1395-1721): same search (11 alphas, loss = mean((out - out_actual)^2)),
  with the weight side of every alpha done by one fused HIP pass (``block_quant_dynamic``:
  ``W * s`` rounded to the weight dtype, in-kernel block amax, INT-n qdq) instead of the
  reference's multiply + two reductions + qdq; per-alpha losses stay on the device and are read
  once per layer (the reference does one host ``float()`` per alpha).
"""

from __future__ import annotations

import math
import os
import warnings
import weakref
from collections.abc import Callable

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from modelopt_amd._ext import ops as _ops
from modelopt_amd.torch.utils.distributed import DistributedProcessGroup, fixed_order_sum_many

from .conversion import set_quantizer_by_cfg_context
from .nn.modules.quant_module import QuantModule
from .nn.modules.tensor_quantizer import SequentialQuantizer, StaticBlockScaleQuantizer, TensorQuantizer
from .utils import core_utils as quant_utils
from .utils.names import is_quantized_linear

__all__ = [
    "apply_pre_quant_scale_and_smooth",
    "awq",
    "awq_lite",
    "enable_stats_collection",
    "finish_stats_collection",
    "max_calibrate",
    "promote_static_block_weight_quantizers",
    "sync_amax_packed",
    "weight_only_quantize",
]

ForwardLoop = Callable[[nn.Module], None]


def enable_stats_collection(model: nn.Module):
    """Quant off, calib on for every enabled quantizer (reference :1128-1141)."""
    from .calib.max import new_collect_epoch

    new_collect_epoch()
    for _, module in model.named_modules():
        if isinstance(module, TensorQuantizer) and not module._disabled:
            if module._use_constant_amax or module._constant_amax is not None:
                module.disable_quant()
                continue
            if module._calibrator is not None:
                module.disable_quant()
                module.enable_calib()
            else:
                module.disable()


def finish_stats_collection(model: nn.Module, method: str | None = None, **kwargs):
    """Load amax from the calibrators, quant on, calib off (reference :1144-1167)."""
    from .calib.max import MaxCalibrator

    # one batched NaN/inf check for every max calibrator instead of a host sync per quantizer
    MaxCalibrator.validate_many(
        getattr(m, "_calibrator", None) for m in model.modules() if isinstance(m, TensorQuantizer)
    )
    for _, module in model.named_modules():
        if not isinstance(module, TensorQuantizer) or module._disabled:
            continue
        if module._use_constant_amax or module._constant_amax is not None:
            module.enable_quant()
            continue
        cal = getattr(module, "_calibrator", None)
        if cal and not getattr(module, "_dynamic", False):
            if method is None and not kwargs and type(cal) is MaxCalibrator and type(module) is TensorQuantizer:
                # load_calib_amax's steps with the amax computed once (its fp32 -> dtype cast is a
                # fresh tensor: adopted without the setter's copy)
                amax = cal.compute_amax()
                if amax is not None:
                    module._adopt_calib_amax(amax, cal)
            elif method is not None:
                if cal.compute_amax(method, **kwargs) is not None:
                    module.load_calib_amax(method, **kwargs)
            elif cal.compute_amax(**kwargs) is not None:
                module.load_calib_amax(**kwargs)
        module.enable_quant()
        module.disable_calib()


def weight_only_quantize(model: nn.Module):
    """Run every weight quantizer once on its weight (reference :187-199)."""
    seen = set()
    for module in model.modules():
        if module in seen:
            continue
        if isinstance(module, QuantModule):
            for weight, weight_quantizer in module.iter_weights_for_calibration():
                weight_quantizer(weight)
        seen.add(module)


def _iter_leaf_quantizers(q):
    if isinstance(q, SequentialQuantizer):
        for s in q:
            yield from _iter_leaf_quantizers(s)
        return
    yield q


def sync_amax_packed(quantizers: list[TensorQuantizer], group: DistributedProcessGroup) -> int:
    """One all_reduce(MAX) over all quantizers' ``_amax`` (grouped by device).

    Packs every amax (any dtype, exact in fp32) into one fp32 buffer, reduces once, unpacks.
    Returns the number of collectives issued."""
    if not group.is_initialized():
        return 0
    qs = [q for q in quantizers if getattr(q, "_amax", None) is not None]
    by_dev: dict[torch.device, list[TensorQuantizer]] = {}
    for q in qs:
        by_dev.setdefault(q._amax.device, []).append(q)
    backend = dist.get_backend(group.group)
    n = 0
    for dev, lst in sorted(by_dev.items(), key=lambda kv: str(kv[0])):
        flat = torch.cat([q._amax.detach().reshape(-1).to(torch.float32) for q in lst])
        if backend == "nccl" and flat.device.type != "cuda":
            continue
        if backend == "gloo" and flat.device.type != "cpu":
            flat_c = flat.cpu()
            dist.all_reduce(flat_c, op=dist.ReduceOp.MAX, group=group.group)
            flat = flat_c.to(dev)
        else:
            dist.all_reduce(flat, op=dist.ReduceOp.MAX, group=group.group)
        n += 1
        off = 0
        for q in lst:
            k = q._amax.numel()
            q._amax.data.copy_(flat[off : off + k].view_as(q._amax).to(q._amax.dtype))
            off += k
    return n


def promote_static_block_weight_quantizers(model: nn.Module) -> int:
    """INT static-block weight quantizers -> StaticBlockScaleQuantizer (core_utils.py:1077-1150)."""
    converted = 0
    for _, module in list(model.named_modules()):
        if not isinstance(module, QuantModule):
            continue
        for _, q in module.iter_weights_for_calibration():
            if isinstance(q, SequentialQuantizer):
                if len(q) == 0:
                    continue
                q = q[0]
            if not isinstance(q, TensorQuantizer) or not q.is_enabled or not q.is_static_block_quant:
                continue
            if q.amax is None:
                continue
            if q.is_nvfp4_static:
                # two-level NVFP4: the global amax is the max of the per-block amax
                # (reference core_utils.py:1129-1143, no shared-state groups)
                promoted = isinstance(q, StaticBlockScaleQuantizer)
                if not q.amax.is_meta:
                    StaticBlockScaleQuantizer.from_tensor_quantizer(q, global_amax=q.amax.detach().float().amax())
                    converted += 0 if promoted else 1
                continue
            if isinstance(q._num_bits, int) and not isinstance(q, StaticBlockScaleQuantizer):
                StaticBlockScaleQuantizer.from_tensor_quantizer(q)
                converted += 1
    return converted


@torch.no_grad()
def max_calibrate(
    model: nn.Module,
    forward_loop: ForwardLoop | None = None,
    distributed_sync=True,
    sync_expert_weight_amax=False,
    shared_states=None,
    skip_forward_without_activation_calib: bool = False,
):
    """Max calibration (reference :311-498)."""
    enable_stats_collection(model)
    weight_only_quantize(model)
    if forward_loop is not None:
        forward_loop(model)
    with quant_utils.gc_paused():
        finish_stats_collection(model)

    for _, module in model.named_modules():
        if hasattr(module, "layer_sync_moe_local_experts_amax"):
            module.layer_sync_moe_local_experts_amax(sync_weight_amax=sync_expert_weight_amax)

    if distributed_sync:
        # DP sync: one packed all_reduce per process group instead of one per quantizer
        groups: dict[int, tuple[DistributedProcessGroup, list]] = {}
        for _, module in model.named_modules():
            if isinstance(module, QuantModule) and module.parallel_state is not None:
                g = module.parallel_state.data_parallel_group
                for child in module.children():
                    if isinstance(child, (TensorQuantizer, SequentialQuantizer)):
                        groups.setdefault(id(g.group) if g.group is not None else 0, (g, []))[1].extend(
                            _iter_leaf_quantizers(child)
                        )
                    elif isinstance(child, nn.ModuleList):
                        for c in child:
                            if isinstance(c, (TensorQuantizer, SequentialQuantizer)):
                                groups.setdefault(id(g.group) if g.group is not None else 0, (g, []))[1].extend(
                                    _iter_leaf_quantizers(c)
                                )
        for g, qs in groups.values():
            seen, uniq = set(), []
            for q in qs:
                if id(q) not in seen:
                    seen.add(id(q))
                    uniq.append(q)
            sync_amax_packed(uniq, g)
    promote_static_block_weight_quantizers(model)


# ------------------------------------------------------------------------------------------------
# AWQ-lite
# ------------------------------------------------------------------------------------------------


def _get_awq_quantizer_block_size(weight: torch.Tensor, wq) -> int | None:
    """Block size of the weight quantizer (reference :1943-1952)."""
    if isinstance(wq, SequentialQuantizer):
        wq = wq[0]
    bs = wq.block_sizes
    if bs is None:
        return None
    return bs.get(-1, None) or bs.get(weight.dim() - 1, None)


def get_weight_scale(weight, block_size=None):
    """mean_rows(|W| / (block amax + tiny)) in the weight dtype, fp32 out (reference :1453-1469)."""
    org_shape = weight.shape
    slice_after_padding = None
    if block_size:
        if org_shape[-1] % block_size != 0:
            slice_after_padding = slice(org_shape[-1])
            weight = F.pad(weight, (0, block_size - org_shape[-1] % block_size), "constant", 0)
            org_shape = weight.shape
        weight = weight.contiguous().view(-1, block_size)
    weight_abs = weight.abs()
    weight_abs_amax = weight_abs.amax(dim=1, keepdim=True)
    scale = weight_abs / (weight_abs_amax + torch.finfo(weight.dtype).tiny)
    scale = scale.view(org_shape)
    if slice_after_padding is not None:
        scale = scale[..., slice_after_padding]
    if _cpu_order_ok(scale):
        # the mean in the reference CPU run's summation order (csrc/mtq_awq_scale.hip): torch's
        # device mean sums in another order and multiplies by 1/N
        return _ops().col_mean(scale.reshape(-1, scale.shape[-1]), False)
    return scale.mean(0).to(torch.float32)


def get_act_scale(x):
    """mean_tokens(|x|) in fp32 (reference :1471-1472)."""
    if _cpu_order_ok(x):
        return _ops().col_mean(x, True)  # |x| and the CPU summation order in one pass
    return x.abs().contiguous().view(-1, x.shape[-1]).mean(0).to(torch.float32)


def _cpu_order_ok(t) -> bool:
    """The AWQ statistics of a device tensor go through the kernels that reproduce the reference's
    CPU operation order bit for bit (mtq_col_mean / mtq_awq_scale_table)."""
    return (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and t.dim() >= 1 and t.numel() > 0)


def _true_div(t: torch.Tensor, n) -> torch.Tensor:
    """``t / n`` for a Python number ``n`` as the reference's CPU run computes it (a correctly
    rounded division): torch on the GPU turns a division by a host scalar into a multiplication
    by its reciprocal, which is 1 ulp off on some elements."""
    if isinstance(t, torch.Tensor) and t.is_cuda and t.is_floating_point():
        return t / torch.tensor(n, dtype=t.dtype, device=t.device)
    return t / n


# The linears that read one tensor (q/k/v_proj, gate/up_proj) each take its act scale in the caching
# pass; the last result is kept for the same tensor object at the same version (the reference
# recomputes it per linear: same ops, same value).
_act_scale_memo = [None, None, None]  # weakref to the tensor, its _version, the act scale


def _act_scale_shared(x):
    if x.is_inference():
        # inference tensors (torch.inference_mode) carry no version counter to key the memo on
        return get_act_scale(x)
    ref, ver, val = _act_scale_memo
    if ref is not None and ref() is x and ver == x._version:
        return val
    val = get_act_scale(x)
    _act_scale_memo[:] = [weakref.ref(x), x._version, val]
    return val


def _act_scale_memo_clear():
    _act_scale_memo[:] = [None, None, None]


def get_scale(x_max, w_max, alpha, tensor_parallel_group=None):
    """AWQ scale for one alpha (reference :1474-1487)."""
    if _cpu_order_ok(x_max) and x_max.dtype == torch.float32:
        scales = _scale_table(x_max, w_max, [alpha])[0]
        if tensor_parallel_group is not None and tensor_parallel_group.is_initialized():
            dist.all_reduce(scales, op=dist.ReduceOp.SUM, group=tensor_parallel_group.group)
            scales /= tensor_parallel_group.world_size()
        return scales
    scales = (
        (x_max.pow(alpha) / (w_max.to(x_max.device).pow(1 - alpha) + torch.finfo(torch.float32).tiny))
        .clamp(min=1e-4, max=1e4)
        .view(-1)
    )
    scales = (scales / (scales.max() * scales.min()).sqrt()).view(-1)
    if tensor_parallel_group is not None and tensor_parallel_group.is_initialized():
        dist.all_reduce(scales, op=dist.ReduceOp.SUM, group=tensor_parallel_group.group)
        scales /= tensor_parallel_group.world_size()
    return scales


def _scale_table(x_max, w_max, alphas):
    """``torch.stack([get_scale(x_max, w_max, a) for a in alphas])`` in ~30 launches instead of
    ~11 per alpha: the two pows stay per alpha (torch special-cases some exponents: 0 fills ones,
    0.5 is sqrt, 1 copies), every other step runs once on the [G, K] stack -- the same IEEE
    operations on the same elements, and max / min are exact, so the table is bit-identical
    (tests/test_awq_scale_table.py).  The search tables of every linear are built in the first
    search batch, where ~110 small host-issued ops per linear held the GPU back by ~0.6 s."""
    w = w_max.to(x_max.device)
    if _cpu_order_ok(x_max) and x_max.dtype == torch.float32 and w.dtype == torch.float32:
        # one launch for every alpha, with the pow of the reference's CPU run (ATen's vectorised
        # powf and its special exponents, csrc/mtq_awq_scale.hip): bit-identical rows
        e_num = torch.tensor([float(a) for a in alphas], dtype=torch.float64)
        e_den = torch.tensor([1 - a for a in alphas], dtype=torch.float64)
        return _ops().awq_scale_table(x_max.reshape(-1), w.reshape(-1), e_num, e_den)
    num = torch.stack([x_max.pow(a) for a in alphas])
    den = torch.stack([w.pow(1 - a) for a in alphas])
    scales = (num / (den + torch.finfo(torch.float32).tiny)).clamp(min=1e-4, max=1e4)
    norm = (scales.amax(dim=1, keepdim=True) * scales.amin(dim=1, keepdim=True)).sqrt()
    return scales / norm


class _AWQLiteHelper:
    cache_mode: bool = False
    _live: "weakref.WeakSet[_AWQLiteHelper]" = weakref.WeakSet()

    def __init__(self, module, name, alpha_step):
        _AWQLiteHelper._live.add(self)
        self.name = name
        self.act_scale = 0.0
        self.num_cache_steps = 0
        self.num_search_steps = 0
        self.block_size = _get_awq_quantizer_block_size(module.weight, module.weight_quantizer)
        self.weight_scale = get_weight_scale(module.weight, self.block_size)
        self.alphas = [k.item() for k in torch.arange(0, 1.0 + alpha_step, alpha_step)]
        self.loss = torch.zeros(len(self.alphas), device=module.weight.device, dtype=torch.float32)
        self.best_scale = None
        self.best_alpha = None
        self.is_input_quantized = module.input_quantizer.is_enabled
        self.num_tokens = 0
        self.module = module
        self.is_enabled = True
        self.dp_group = None  # set when act_scale is synced over a DP group

    def setup(self):
        module = self.module
        module._forward_no_awq = module.forward
        module.forward = _awq_forward.__get__(module, type(module))
        if module.input_quantizer.is_enabled:
            module.input_quantizer.disable()
            if module.input_quantizer.axis not in [None, -1]:
                self.is_enabled = False
                return
            module.input_quantizer.axis = -1

    def cleanup(self):
        module = self.module
        if "forward" in module.__dict__:
            del module.__dict__["forward"]
        if "_forward_no_awq" in module.__dict__:
            del module.__dict__["_forward_no_awq"]


def _weight_qdq_fast_path(wq: TensorQuantizer, weight: torch.Tensor):
    """Whether the weight quantizer's dynamic-amax static-block INT qdq can run fused."""
    bs = wq.block_sizes or {}
    blk = bs.get(-1) or bs.get(weight.dim() - 1)
    return (
        isinstance(wq, TensorQuantizer)
        and wq.is_enabled
        and wq.fake_quant
        and wq.backend is None
        and isinstance(wq._num_bits, int)
        and wq.is_static_block_quant
        and not hasattr(wq, "_amax")
        and blk in (32, 64, 128, 256)
        and len([k for k in bs if isinstance(k, int)]) == 1
        and weight.dim() == 2
        and weight.shape[-1] % blk == 0
        and weight.is_cuda
        and weight.dtype in (torch.bfloat16, torch.float16, torch.float32)
    ), blk


_FAST_DTYPES = (torch.bfloat16, torch.float16, torch.float32)


def _mse_fast(out, ref) -> bool:
    return (
        isinstance(out, torch.Tensor) and isinstance(ref, torch.Tensor) and out.is_cuda
        and out.dtype == ref.dtype and out.dtype in _FAST_DTYPES and out.shape == ref.shape
        and out.numel() > 0
    )


# Fused AWQ search on MFMA (csrc/mtq_awq_gemm.hip): used for linears with at most this many output
# features or with at least as many output as input features, where it beats the library path
# (r06, the one-wave-per-SIMD kernel, scripts/bench_awq_gemm.py at Llama-3-8B shapes: k/v, q/o,
# gate/up fused; down_proj -- K 14336 > N 4096, whose x * (1/s) pass alone is 0.6 ms of the fused
# call -- keeps the library); the others run one hipBLASLt GEMM per alpha between one x * (1/s)
# pass and one loss pass for all alphas.
# MTQ_AMD_AWQ_FUSED: "auto" (default), "always" (fused kernel for every width), "library" (the
# hipBLASLt path for every width), "never" (the reference's per-alpha loop, no fast path).
_AWQ_FUSED_MAX_N = 2048
_AWQ_FUSED_MAX_G = 64
_AWQ_FUSED = os.environ.get("MTQ_AMD_AWQ_FUSED", "auto")
_AWQ_FUSED_CHOICES = ("auto", "always", "library", "never")


def _awq_use_fused(m_rows: int, n_out: int, k_in: int, n_alpha: int, mode: str | None = None) -> bool:
    """Route one linear's AWQ search: the fused MFMA kernel (mtq_awq_search_gemm) or the batched
    hipBLASLt path.  The kernel's limits: G <= 64 alphas, 32-bit element offsets.  "auto": fused
    where N <= 2048 or K <= N (measured faster there, DESIGN.md §4e r06 -- k/v, q/o, gate/up of
    Llama-3-8B; down_proj, K > N, keeps the library)."""
    mode = _AWQ_FUSED if mode is None else mode
    ok = n_alpha <= _AWQ_FUSED_MAX_G and m_rows * k_in < 2**31 and n_out * k_in < 2**31
    return ok and (mode == "always" or (mode == "auto" and (n_out <= _AWQ_FUSED_MAX_N or k_in <= n_out)))


def _check_awq_fused() -> None:
    """Validate MTQ_AMD_AWQ_FUSED where it is used (awq_lite); a misspelt value only warns at
    import, so workflows that never reach the AWQ search are not broken by it."""
    if _AWQ_FUSED not in _AWQ_FUSED_CHOICES:
        raise ValueError(f"MTQ_AMD_AWQ_FUSED={_AWQ_FUSED!r}: expected auto, always, library or never")


if _AWQ_FUSED not in _AWQ_FUSED_CHOICES:
    warnings.warn(f"MTQ_AMD_AWQ_FUSED={_AWQ_FUSED!r}: expected auto, always, library or never; "
                  "awq_lite will raise", stacklevel=1)
# Budget for keeping every alpha's quantised weight [11, N, K] across the search batches (it does
# not change between batches; the reference recomputes it per batch): a fraction of the HBM free
# when the search pass starts (Llama-3-8B: 154 GB of 288 GB).
_AWQ_WQ_CACHE_FRACTION = float(os.environ.get("MTQ_AMD_AWQ_WQ_CACHE_FRACTION", "0.6"))
_awq_wq_budget = [0]


def _awq_search_tables(helper, dtype):
    """Per-alpha scales of the whole search, [G, K] each: pre_quant_scale of the weight side and
    of the input side, exactly as the per-alpha code computes them (get_scale, then
    ``(1 / s).to(dtype)`` / ``s.to(dtype)``), stacked once per linear."""
    if getattr(helper, "_tables", None) is None:
        s = _scale_table(helper.act_scale, helper.weight_scale, helper.alphas)
        helper._tables = ((1 / s).to(dtype), s.to(dtype))
        helper._scale_rows = s  # fp32: the best alpha's row is the final scale (get_scale's bits)
    return helper._tables


def _awq_wq_all(self, helper, pqs_w, blk):
    wq = getattr(helper, "_wq_all", None)
    if wq is not None:
        return wq
    q = self.weight_quantizer
    wq = _ops().block_quant_dynamic_multi(self.weight.detach(), pqs_w, blk, q._num_bits, q._unsigned,
                                          q._narrow_range)
    nbytes = wq.numel() * wq.element_size()
    if nbytes <= _awq_wq_budget[0]:
        _awq_wq_budget[0] -= nbytes
        helper._wq_all = wq
    return wq


def _awq_search_fast(self, helper, input, out_act, blk) -> bool:
    """All alphas of one search batch with the weight side computed once per linear; the GEMM +
    loss either fused on MFMA (narrow linears) or per alpha on hipBLASLt.  False when the
    module / tensors do not qualify (the generic per-alpha path then runs)."""
    w = self.weight
    if not (
        isinstance(out_act, torch.Tensor) and out_act.is_cuda and out_act.dtype == w.dtype
        and input.is_cuda and input.dtype == w.dtype and w.dtype in (torch.bfloat16, torch.float16)
        and not self.output_quantizer.is_enabled and not self.input_quantizer.is_enabled
        and input.shape[-1] % 64 == 0 and w.shape[0] % 8 == 0
        and out_act.shape[-1] == w.shape[0] and out_act.numel() // w.shape[0] == input.numel() // w.shape[1]
    ):
        return False
    sinv, pqs_w = _awq_search_tables(helper, w.dtype)
    wq = _awq_wq_all(self, helper, pqs_w, blk)
    ops = _ops()
    bias = self.bias.detach() if self.bias is not None else None
    x2 = input.reshape(-1, input.shape[-1])
    n_out, k_in, n_alpha = w.shape[0], w.shape[1], len(helper.alphas)
    if _awq_use_fused(x2.shape[0], n_out, k_in, n_alpha):
        ops.awq_search_gemm(x2, sinv, wq, bias, out_act.reshape(-1, w.shape[0]), helper.loss)
    elif n_alpha <= 16:
        # wide linears: x * (1/s) for every alpha in one pass, one hipBLASLt GEMM per alpha into
        # slices of one [G, M, N] output (bias in its fp32 epilogue, one rounding, as F.linear;
        # per-alpha torch.mm, the GEMM F.linear itself uses: torch.bmm with the transposed
        # [G, K, N] weight view faulted the GPU in hipBLASLt on ROCm 7 at [11, 8192, 4096] x
        # [11, 4096, 4096]), all losses in one pass that reads out_actual once.  Serial on one
        # stream: the prescale and loss passes on a side stream beside the GEMMs were measured
        # 5-30 % slower (they displace GEMM workgroups; profiles/r04/awq/overlap_ab_r04e.json).
        try:
            xs = ops.awq_prescale(x2, sinv)
            out = torch.empty((xs.shape[0], xs.shape[1], w.shape[0]), dtype=w.dtype, device=w.device)
        except torch.cuda.OutOfMemoryError:
            # the cached [G, N, K] weights of the other linears hold the HBM: drop them, retry
            xs = None
            _awq_release_wq_caches()
            xs = ops.awq_prescale(x2, sinv)
            out = torch.empty((xs.shape[0], xs.shape[1], w.shape[0]), dtype=w.dtype, device=w.device)
        for ai in range(xs.shape[0]):
            if bias is None:
                torch.mm(xs[ai], wq[ai].t(), out=out[ai])
            else:
                torch.addmm(bias, xs[ai], wq[ai].t(), out=out[ai])
        del xs
        ops.awq_mse_multi(out, out_act.reshape(-1, w.shape[0]), helper.loss)
    else:
        for ai in range(len(helper.alphas)):
            out = F.linear(ops.mul_cols(x2, sinv[ai]), wq[ai], bias)
            ops.mse_accumulate(out, out_act.reshape(-1, w.shape[0]), helper.loss, ai)
    return True


def _awq_forward(self, input, *args, **kwargs):
    """Patched QuantLinear forward during AWQ-lite (reference :1513-1560)."""
    helper = self.awq_lite
    self.weight_quantizer.disable()
    if hasattr(self.input_quantizer, "_pre_quant_scale"):
        delattr(self.input_quantizer, "_pre_quant_scale")
    if hasattr(self.weight_quantizer, "_pre_quant_scale"):
        delattr(self.weight_quantizer, "_pre_quant_scale")
    out_actual = self._forward_no_awq(input, *args, **kwargs)
    self.weight_quantizer.enable()

    if input.numel() == 0 or not helper.is_enabled:
        return out_actual

    if _AWQLiteHelper.cache_mode:
        helper.act_scale = helper.act_scale + _act_scale_shared(self.input_quantizer(input))
        helper.num_cache_steps += 1
        helper.num_tokens += input.numel() / input.shape[-1]
        if helper.is_input_quantized:
            with set_quantizer_by_cfg_context(self.input_quantizer, [{"quantizer_name": "*", "enable": True}]):
                max_calibrate(self.input_quantizer, lambda q: q(input), False)
        return out_actual

    fast, blk = _weight_qdq_fast_path(self.weight_quantizer, self.weight)
    out_act = out_actual[0] if isinstance(out_actual, tuple) else out_actual
    if (
        fast and not args and not kwargs and type(self)._original_cls is nn.Linear
        and _AWQ_FUSED != "never" and _awq_search_fast(self, helper, input, out_act, blk)
    ):
        helper.num_search_steps += 1
        return out_actual
    ops = _ops()
    x_fast = (
        input.is_cuda and input.dtype == self.weight.dtype and input.dtype in _FAST_DTYPES
        and input.shape[-1] % (16 // input.element_size()) == 0
    )
    for ai, alpha in enumerate(helper.alphas):
        awq_scale = get_scale(helper.act_scale, helper.weight_scale, alpha, None)
        pqs_in = (1 / awq_scale).to(self.weight.dtype)
        pqs_w = awq_scale.to(self.weight.dtype)
        if fast and not args and not kwargs and type(self)._original_cls is nn.Linear:
            # fused: qdq(W * s) in one HIP pass, x * (1/s) as the input quantizer would apply it
            wq = ops.block_quant_dynamic(
                self.weight.detach(), pqs_w, blk, self.weight_quantizer._num_bits,
                self.weight_quantizer._unsigned, self.weight_quantizer._narrow_range,
            )
            xs = ops.mul_cols(input, pqs_in) if x_fast else input * pqs_in
            out = F.linear(self.input_quantizer(xs), wq, self.bias)
            out = self.output_quantizer(out)
        else:
            self.input_quantizer.pre_quant_scale = pqs_in
            self.weight_quantizer.pre_quant_scale = pqs_w
            out = self._forward_no_awq(input, *args, **kwargs)
        out = out[0] if isinstance(out, tuple) else out
        if _mse_fast(out, out_act):
            # (out - out_act).float().pow(2).mean() in one HIP pass (model_calib.py:1494)
            ops.mse_accumulate(out, out_act, helper.loss, ai)
        else:
            helper.loss[ai] += (out - out_act).float().pow(2).mean()
    helper.num_search_steps += 1
    return out_actual


@torch.no_grad()
def apply_pre_quant_scale_and_smooth(linear: nn.Module, pre_quant_scale: torch.Tensor | None = None,
                                     _distributed_sync: bool = True):
    """Fold 1/pre_quant_scale into the weight and re-calibrate it (reference :1209-1270).

    ``_distributed_sync=False`` (awq_lite): the folded weights are bit-identical on every DP rank
    by construction (act_scale and losses are synced before the choice), so the reference's
    per-linear weight-amax all_reduce(MAX) is an identity and is skipped."""
    assert is_quantized_linear(linear), "Only quantized linear modules are supported"
    assert linear.input_quantizer.pre_quant_scale is None, "pre_quant_scale should be None first!"
    if pre_quant_scale is None:
        pre_quant_scale = getattr(linear.input_quantizer, "_pre_quant_scale", None)
    assert pre_quant_scale is not None, "pre_quant_scale should be provided or already set"
    assert torch.all(pre_quant_scale > 0), "pre_quant_scale should be positive"
    pre_quant_scale = pre_quant_scale.to(torch.float32)
    linear.input_quantizer._enable_pre_quant_scale = True
    linear.input_quantizer.pre_quant_scale = pre_quant_scale.to(linear.weight.dtype)
    inv_scale = 1.0 / pre_quant_scale
    # _apply_weight_pre_quant_scale with folding (reference :1209-1223)
    linear.weight.data.copy_(
        (linear.weight * inv_scale.to(linear.weight.device).squeeze()[None, :]).to(linear.weight.dtype)
    )
    linear.weight_quantizer.reset_amax()
    max_calibrate(linear, lambda lin: lin.weight_quantizer(lin.weight), distributed_sync=_distributed_sync)
    if linear.input_quantizer.amax is not None:
        assert hasattr(linear.input_quantizer, "_amax_for_smoothing")
        dev, dt = linear.weight.device, linear.weight.dtype
        a = linear.input_quantizer._amax_for_smoothing.to(device=dev, dtype=dt)
        linear.input_quantizer.amax = (a * pre_quant_scale.to(dev)).amax().to(dt)


def _awq_dp_groups(awq_modules):
    """The AWQ linears grouped by their initialised data-parallel group, in module order (the
    same on every rank); linears without one are returned under key None."""
    groups: dict = {}
    for name, module in awq_modules:
        g = module.parallel_state.data_parallel_group if module.parallel_state is not None else None
        key = None if g is None or not g.is_initialized() else (id(g.group) if g.group is not None else 0)
        groups.setdefault(key, (g, []))[1].append((name, module))
    return groups


def _awq_sync_act_scale(awq_modules):
    """After the caching pass: act_scale = mean over the cache steps, NaN check, DP average.

    Reference :1595-1629 issues, per linear, an ``all_gather_object`` of a NaN flag and an
    ``all_reduce(AVG)`` of act_scale, both gated on the rank-local ``num_cache_steps > 0`` (a
    linear that saw tokens on one rank only -- an MoE expert -- would enter the collectives on
    that rank alone).  Here every linear of a DP group contributes ``[act_scale, nan, present]``
    (zeros when it saw no tokens) to ONE fixed-order sum (``fixed_order_sum_many``: one all_gather
    per group, independent of the number of linears), and every rank takes the same decision:
    disabled when a rank saw NaN or no rank saw tokens, otherwise act_scale = sum of the ranks that
    saw tokens / their count (the reference's AVG when all ranks saw tokens), rounded back to the
    act_scale dtype."""
    for key, (g, mods) in _awq_dp_groups(awq_modules).items():
        if key is None:
            for _, module in mods:
                h = module.awq_lite
                if h.num_cache_steps == 0:
                    h.is_enabled = False
                    continue
                module._if_calib = True
                h.act_scale = _true_div(h.act_scale, h.num_cache_steps)
                if bool(torch.isnan(h.act_scale).any() or torch.isnan(h.weight_scale).any()):
                    h.is_enabled = False
            continue
        parts = []
        for _, module in mods:
            h = module.awq_lite
            k = module.weight.shape[1]
            dev = h.weight_scale.device
            if h.num_cache_steps > 0:
                a = _true_div(h.act_scale, h.num_cache_steps).reshape(-1)
                nan = (torch.isnan(a).any() | torch.isnan(h.weight_scale).any()).reshape(1)
                present = torch.ones(1, device=dev)
            else:
                a = torch.zeros(k, device=dev)
                nan = torch.zeros(1, device=dev)
                present = torch.zeros(1, device=dev)
            parts += [a.to(device=dev, dtype=torch.float32), nan.to(torch.float32), present]
        summed = fixed_order_sum_many(parts, g)
        for i, (_, module) in enumerate(mods):
            h = module.awq_lite
            a, nan, present = summed[3 * i : 3 * i + 3]
            n_present, n_nan = float(present), float(nan)  # host reads of one gathered buffer
            if n_present == 0 or n_nan > 0:
                h.is_enabled = False
                continue
            module._if_calib = True
            dtype = h.act_scale.dtype if isinstance(h.act_scale, torch.Tensor) else torch.float32
            # fixed_order_sum_many returns every slice on the first linear's device: back to this
            # linear's (a model spread over several GPUs by device_map)
            h.act_scale = _true_div(a, n_present).to(device=h.weight_scale.device, dtype=dtype)
            h.dp_group = g
            h._dp_cache_steps = n_present


def _awq_sync_losses(awq_modules):
    """After the search pass: per-alpha losses summed over the DP ranks in rank order (one
    collective per group), and the reference's "search pass missed this linear" check
    (:1661-1671) taken on the group-wide counts so every rank disables the same linears.

    Divergence from the reference (which keeps each rank's local losses, so ranks with different
    data can pick different alphas and end with different weights): every rank picks the alpha a
    single process over all the data would."""
    for key, (g, mods) in _awq_dp_groups(awq_modules).items():
        if key is None:
            searched = {name: module.awq_lite.num_search_steps > 0 for name, module in mods}
            cached = {name: module.awq_lite.num_cache_steps > 0 for name, module in mods}
        else:
            parts = []
            for _, module in mods:
                h = module.awq_lite
                dev = h.loss.device
                parts += [h.loss, torch.full((1,), float(h.num_search_steps > 0), device=dev),
                          torch.full((1,), float(h.num_cache_steps > 0), device=dev)]
            summed = fixed_order_sum_many(parts, g)
            searched, cached = {}, {}
            for i, (name, module) in enumerate(mods):
                h = module.awq_lite
                loss, s, c = summed[3 * i : 3 * i + 3]
                h.loss = loss.to(h.loss.device)
                searched[name], cached[name] = float(s) > 0, float(c) > 0
        for name, module in mods:
            h = module.awq_lite
            if cached[name] and not searched[name] and h.is_enabled:
                h.is_enabled = False
                warnings.warn(
                    f"awq_lite: Calling `forward_loop(model)` the second time did not forward data through the {name}."
                )


def _awq_wq_cache_budget() -> int:
    """HBM for the [G, N, K] quantised-weight cache of the search: a fraction of the free HBM,
    divided among the processes that share this device (ranks of one node on fewer GPUs: the
    2-rank tests and the C4 pipeline rehearsal on one MI355X), each of which would otherwise claim
    the same free memory."""
    free = torch.cuda.mem_get_info()[0]
    local = os.environ.get("LOCAL_WORLD_SIZE")
    if local:
        local = int(local)
    else:  # spawned workers without torchrun's env: one node assumed
        local = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    per_dev = max(1, -(-local // max(1, torch.cuda.device_count())))
    return int(free * _AWQ_WQ_CACHE_FRACTION / per_dev)


def _awq_release_wq_caches():
    """Drop every cached [G, N, K] search weight (after an allocation failure in the search)."""
    for h in list(_AWQLiteHelper._live):
        h._wq_all = None
    _awq_wq_budget[0] = 0  # no new caching after a failure
    torch.cuda.empty_cache()


@torch.no_grad()
def awq_lite(model: nn.Module, forward_loop: ForwardLoop, alpha_step: float = 0.1, debug: bool = False, **kwargs):
    """AWQ-lite scale search (reference :1395-1721)."""
    _check_awq_fused()
    if forward_loop is None:
        warnings.warn("forward_loop must be provided for awq_lite; skipping awq_lite")
        return
    for name, module in list(model.named_modules()):
        if is_quantized_linear(module) and module.weight_quantizer.is_enabled:
            module.awq_lite = _AWQLiteHelper(module, name, alpha_step)
            module.awq_lite.setup()

    _AWQLiteHelper.cache_mode = True
    enable_stats_collection(model)
    try:
        forward_loop(model)
    finally:
        _act_scale_memo_clear()  # the last act scale is not kept alive past the caching pass
    with set_quantizer_by_cfg_context(model, [{"quantizer_name": "*weight_quantizer", "enable": False}]):
        max_calibrate(model, lambda m: None, distributed_sync=True)
    finish_stats_collection(model)

    awq_modules = [
        (name, module) for name, module in model.named_modules()
        if is_quantized_linear(module) and isinstance(getattr(module, "awq_lite", None), _AWQLiteHelper)
    ]
    _awq_sync_act_scale(awq_modules)

    _AWQLiteHelper.cache_mode = False
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
        _awq_wq_budget[0] = _awq_wq_cache_budget()
    forward_loop(model)
    _awq_wq_budget[0] = 0
    for _, module in model.named_modules():
        h = getattr(module, "awq_lite", None)
        if isinstance(h, _AWQLiteHelper):
            h._wq_all = None
            h._tables = None
    _awq_sync_losses(awq_modules)

    def postprocess(module, name):
        h = module.awq_lite
        if h.is_enabled:
            losses = h.loss.tolist()  # one host read per layer
            # the reference's loss dict of floats (update_best_params, :1497-1511)
            h.loss = dict(zip(h.alphas, losses))
            h.best_alpha = min(h.loss, key=h.loss.get)
            rows = getattr(h, "_scale_rows", None)
            if rows is not None and rows.shape[0] == len(h.alphas):
                h.best_scale = rows[h.alphas.index(h.best_alpha)].clone()  # == get_scale(best_alpha)
            else:
                h.best_scale = get_scale(h.act_scale, h.weight_scale, h.best_alpha, None)
            h._scale_rows = None
        for q in (module.weight_quantizer, module.input_quantizer):
            if hasattr(q, "_pre_quant_scale"):
                delattr(q, "_pre_quant_scale")
        if h.is_input_quantized:
            if module.input_quantizer.amax is not None:
                act_amax = module.input_quantizer.amax
                module.input_quantizer._amax_for_smoothing = act_amax.cpu()
                module.input_quantizer.reset_amax()
                module.input_quantizer.axis = None
                module.input_quantizer.amax = act_amax.amax()
            module.input_quantizer.enable()
        if h.is_enabled:
            apply_pre_quant_scale_and_smooth(module, 1.0 / h.best_scale, _distributed_sync=False)
        else:
            warnings.warn(f"awq_lite: Disabling for {name}, quantizing with max calibration.")
            max_calibrate(module, lambda m: m.weight_quantizer(m.weight), distributed_sync=False)

    for name, module in model.named_modules():
        if not hasattr(module, "awq_lite"):
            continue
        h = module.awq_lite
        if not h.is_enabled:
            warnings.warn(f"awq_lite: Forcing pre_quant_scale=1 for {name}.")
            max_calibrate(module, lambda m: m.weight_quantizer(m.weight), distributed_sync=False)
            module.input_quantizer._enable_pre_quant_scale = True
            module.input_quantizer.pre_quant_scale = torch.ones(
                module.weight.shape[1], dtype=module.weight.dtype, device=module.weight.device
            )
            if h.is_input_quantized:
                if module.input_quantizer.amax is not None:
                    act_amax = module.input_quantizer.amax
                    module.input_quantizer._amax_for_smoothing = act_amax.cpu()
                    module.input_quantizer.reset_amax()
                    module.input_quantizer.axis = None
                    module.input_quantizer.amax = act_amax.amax()
                module.input_quantizer.enable()
        else:
            postprocess(module, name)
        h.cleanup()
        if "_if_calib" in module.__dict__:
            del module.__dict__["_if_calib"]
        if not debug:
            delattr(module, "awq_lite")


# ---- AWQ-clip (reference model_calib.py:1725-1940) -----------------------------------------------

_CLIP_KERNEL_BLOCKS = (8, 16, 32, 64, 128)


class _AWQClipHelper:
    """Per-linear clip-search state (reference AWQClipHelper, :1746-1783).  The per-shrink losses
    live in one [S, co, n_block] fp32 tensor; ``loss`` is the reference's {shrink: view} dict."""

    def __init__(self, module, min_clip_ratio: float, shrink_step: float):
        self.num_tokens = 0
        self.block_size = _get_awq_quantizer_block_size(module.weight, module.weight_quantizer)
        wq = module.weight_quantizer
        wq.reset_amax()
        enable_stats_collection(wq)
        wq(module.weight)
        finish_stats_collection(wq)
        self.w_amax = wq.amax.clone()
        co, ci = module.weight.shape
        self.shrinks = [round(float(k), 2) for k in torch.arange(min_clip_ratio, 1.0, shrink_step)] + [1.0]
        dev = module.weight.device
        if self.is_per_tensor_clip(module):
            self.loss_tensor = torch.zeros(len(self.shrinks), device=dev)
        else:
            self.loss_tensor = torch.zeros(len(self.shrinks), co, math.ceil(ci / self.block_size), device=dev)
        self.loss = {k: self.loss_tensor[i] for i, k in enumerate(self.shrinks)}
        self.best_clip_val = None
        self.best_loss = None
        self.is_input_quantized = module.input_quantizer.is_enabled
        wq.disable()

    @staticmethod
    def is_per_tensor_clip(module) -> bool:
        q = module.weight_quantizer
        dyn = q.block_sizes is not None and q.block_sizes.get("type", None) == "dynamic" and q.axis is None
        return dyn or (q.axis is None and q.block_sizes is None)


def _awq_clip_update_best_params(module):
    """reference :1785-1797: first strictly smaller loss wins, best = w_amax * shrink."""
    h = module.awq_clip
    h.best_loss = torch.ones_like(h.w_amax) * float("inf")
    h.best_clip_val = torch.zeros_like(h.w_amax)
    for shrink, loss in h.loss.items():
        loss = loss.view_as(h.w_amax)
        idx = loss < h.best_loss
        h.best_loss = torch.where(idx, loss, h.best_loss)
        h.best_clip_val = torch.where(idx, h.w_amax * shrink, h.best_clip_val)


def _clip_kernel_ok(module, inputs) -> bool:
    wq, w = module.weight_quantizer, module.weight
    bs = module.awq_clip.block_size
    return (
        isinstance(wq, TensorQuantizer)
        and type(wq).__name__ in ("TensorQuantizer", "StaticBlockScaleQuantizer")
        and isinstance(wq._num_bits, int)
        and wq.fake_quant
        and wq.backend is None
        and wq.pre_quant_scale is None
        and wq.is_static_block_quant
        and len([k for k in (wq.block_sizes or {}) if isinstance(k, int)]) == 1
        and bs in _CLIP_KERNEL_BLOCKS
        and w.dim() == 2
        and w.is_cuda
        and w.dtype in _FAST_DTYPES
        and inputs.dtype == w.dtype
        and len(module.awq_clip.shrinks) <= 63
        and module.awq_clip.w_amax.numel() == w.shape[0] * math.ceil(w.shape[1] / bs)
    )


def _clip_search(self, inputs, co_bsz=256, max_tokens=16):
    """One clip-search step on a forward (reference :1800-1882)."""
    h = self.awq_clip
    weight = self.weight
    self.weight_quantizer.enable()
    if h.is_per_tensor_clip(self):
        # NVFP4 / per-tensor: only the per-tensor amax is clipped (reference :1804-1815)
        out_actual = inputs @ weight.T
        original_amax = self.weight_quantizer.amax.clone()
        h.num_tokens += inputs.shape[0]
        for i, shrink in enumerate(h.shrinks):
            self.weight_quantizer.amax = original_amax * shrink
            out = inputs @ self.weight_quantizer(weight).T
            if _mse_fast(out, out_actual):
                _ops().mse_accumulate(out, out_actual, h.loss_tensor, i)
            else:
                h.loss_tensor[i] += (out - out_actual).float().pow(2).mean()
        return
    x = inputs.reshape(-1, inputs.shape[-1])
    x = x[0 :: max(1, x.shape[0] // max_tokens)]
    h.num_tokens += x.shape[0]
    bs = h.block_size
    co, ci = weight.shape
    group = self.parallel_state.data_parallel_group if self.parallel_state is not None else None
    dp = group is not None and group.is_initialized()
    if _clip_kernel_ok(self, x):
        # one HIP pass per forward: every (row, block, clip ratio) of the weight at once
        pad = (-ci) % bs
        xs = x.float()
        w = weight.detach()
        if pad:
            xs = F.pad(xs, (0, pad))
            w = F.pad(w, (0, pad))
        xs = xs.contiguous()
        wq = self.weight_quantizer
        shrinks = torch.tensor(h.shrinks, dtype=torch.float32)
        if dp:
            part = torch.empty_like(h.loss_tensor)
            _ops().awq_clip_search(w, xs, h.w_amax, shrinks, part, bs, wq._num_bits, wq._unsigned, wq._narrow_range, False)
            dist.all_reduce(part, op=dist.ReduceOp.SUM, group=group.group)
            part /= group.world_size()
            h.loss_tensor += part
        else:
            _ops().awq_clip_search(w, xs, h.w_amax, shrinks, h.loss_tensor, bs, wq._num_bits, wq._unsigned,
                                   wq._narrow_range, True)
        return
    # the reference's op sequence (any other quantizer), on the device
    if ci % bs != 0:
        weight = F.pad(weight, (0, bs - ci % bs), "constant", 0)
        x = F.pad(x, (0, bs - ci % bs), "constant", 0)
    weight = weight.reshape(co, 1, -1, bs)
    x = x.reshape(1, x.shape[0], -1, bs)
    for b0 in range(0, co, co_bsz):
        sl = slice(b0, min(b0 + co_bsz, co))
        w = weight[sl]
        org_out = (x * w).sum(dim=-1)
        for i, shrink in enumerate(h.shrinks):
            self.weight_quantizer.amax = h.w_amax * shrink
            cur_w = self.weight_quantizer(self.weight)[sl]
            if cur_w.shape[-1] % bs != 0:
                cur_w = F.pad(cur_w, (0, bs - cur_w.shape[-1] % bs), "constant", 0)
            cur_out = (x * cur_w.reshape(w.shape)).sum(dim=-1)
            loss = (cur_out - org_out).float().pow(2).mean(dim=1)
            if dp:
                dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=group.group)
                loss /= group.world_size()
            h.loss_tensor[i, sl] += loss


def _awq_clip_forward(self, input, *args, **kwargs):
    """Patched QuantLinear forward during AWQ-clip (reference :1884-1908)."""
    h = self.awq_clip
    if h.is_input_quantized:
        self.input_quantizer.enable()
        max_calibrate(self.input_quantizer, lambda iq: iq(input))
        self.input_quantizer.disable()
    if input.numel() > 0:
        _clip_search(self, self.input_quantizer(input), h.max_co_batch_size, h.max_tokens_per_batch)
    self.weight_quantizer.disable()
    return self._forward_no_awq(input, *args, **kwargs)


@torch.no_grad()
def awq_clip(model: nn.Module, forward_loop: ForwardLoop, max_co_batch_size: int = 1024,
             max_tokens_per_batch: int = 64, min_clip_ratio: float = 0.5, shrink_step: float = 0.05,
             debug: bool = False, **kwargs):
    """AWQ-clip: per-block clipped amax search on the calibration activations (reference
    :1725-1940).  The block search of a static-block INT weight is one HIP pass per forward
    (``torch.ops.modelopt_amd.awq_clip_search``)."""
    assert forward_loop is not None, "forward_loop must be provided for awq_clip"
    patched = []
    for name, module in model.named_modules():
        if (
            is_quantized_linear(module)
            and module.weight_quantizer.is_enabled
            and module.weight_quantizer.block_sizes is not None
        ):
            module.awq_clip = _AWQClipHelper(module, min_clip_ratio, shrink_step)
            module.awq_clip.max_co_batch_size = max_co_batch_size
            module.awq_clip.max_tokens_per_batch = max_tokens_per_batch
            module._forward_no_awq = module.forward
            module.forward = _awq_clip_forward.__get__(module, type(module))
            patched.append(module)
    enable_stats_collection(model)
    forward_loop(model)
    with set_quantizer_by_cfg_context(model, [{"quantizer_name": "*weight_quantizer", "enable": False}]):
        max_calibrate(model, lambda m: None, distributed_sync=True)
    finish_stats_collection(model)
    for module in patched:
        h = module.awq_clip
        if h.num_tokens > 0:
            _awq_clip_update_best_params(module)
            module.weight_quantizer.amax = h.best_clip_val
            module.weight_quantizer.enable()
            if h.is_input_quantized:
                module.input_quantizer.enable()
        if not debug:
            delattr(module, "awq_clip")
        for k in ("forward", "_forward_no_awq"):
            if k in module.__dict__:
                del module.__dict__[k]


def awq(model: nn.Module, forward_loop: ForwardLoop | None = None, algorithm: str = "awq_lite", **kwargs):
    """AWQ dispatch (reference :1362-1391): awq_lite, awq_clip, or both (awq_full)."""
    with SequentialQuantizer.convert_to_single_quantizer(model):
        if algorithm in ["awq_full", "awq_lite"]:
            awq_lite(model, forward_loop, **{k: v for k, v in kwargs.items() if k in ("alpha_step", "debug")})
        if algorithm in ["awq_full", "awq_clip"]:
            clip_keys = ("max_co_batch_size", "max_tokens_per_batch", "min_clip_ratio", "shrink_step", "debug")
            awq_clip(model, forward_loop, **{k: v for k, v in kwargs.items() if k in clip_keys})
    for _, module in model.named_modules():
        if is_quantized_linear(module) and isinstance(module.weight_quantizer, SequentialQuantizer):
            max_calibrate(module, lambda lin: lin.weight_quantizer(lin.weight))



# ---- MSE weight calibration (reference model_calib.py:639-827) ---------------------------------


def _run_and_load_max_stats(model: nn.Module, forward_loop: ForwardLoop | None = None):
    """Collect + load stats without post-processing (reference :202-209)."""
    enable_stats_collection(model)
    if forward_loop is None:
        weight_only_quantize(model)
    else:
        forward_loop(model)
    finish_stats_collection(model)


def _mse_quant_func(x, amax, quantizer):
    """Fake-quantise ``x`` (the calibrator's block layout) with a candidate ``amax`` (reference
    :639-662): quant on, calib off, fake quant on, the original shape restored around the call."""
    original_amax = quantizer._amax.clone() if hasattr(quantizer, "_amax") else None
    quantizer._amax = amax
    flags = (quantizer._if_quant, quantizer._if_calib, quantizer._fake_quant)
    quantizer._if_quant, quantizer._if_calib, quantizer._fake_quant = True, False, True
    try:
        if hasattr(quantizer, "_original_shape"):
            x = quantizer._reset_to_original_shape(x)
        xq = quantizer(x)
        if hasattr(quantizer, "_block_reshape_size"):
            xq = quantizer._process_for_blockquant(xq)
    finally:
        quantizer._if_quant, quantizer._if_calib, quantizer._fake_quant = flags
        if original_amax is not None:
            quantizer._amax = original_amax
        else:
            delattr(quantizer, "_amax")
    return xq


def _make_weight_mse_calibrator(weight_quantizer, step_size, start_multiplier, stop_multiplier,
                                fp8_scale_sweep, error_func=None, hessian=None):
    """The MSE calibrator for one eligible weight quantizer, or None (reference :665-730)."""
    from functools import partial

    from .calib.mse import MseCalibrator, NVFP4MSECalibrator

    if (
        not isinstance(weight_quantizer, TensorQuantizer)
        or not weight_quantizer.is_enabled
        or weight_quantizer._dynamic
        or weight_quantizer.is_mx_format
        or weight_quantizer._calibrator is None
        or getattr(weight_quantizer, "_amax", None) is None
    ):
        return None
    initial_amax = weight_quantizer._amax.clone().detach()
    axis = weight_quantizer._calibrator._axis
    quant_func = partial(_mse_quant_func, quantizer=weight_quantizer)
    if fp8_scale_sweep:
        if weight_quantizer.backend is None and getattr(weight_quantizer, "is_nvfp4_static", False):
            return NVFP4MSECalibrator(amax=initial_amax, axis=axis, global_amax=weight_quantizer.global_amax,
                                      quant_func=quant_func, error_func=error_func, hessian=hessian)
        return None  # fp8_scale_sweep: only static NVFP4 weights are swept
    return MseCalibrator(amax=initial_amax, axis=axis, step_size=step_size, start_multiplier=start_multiplier,
                         stop_multiplier=stop_multiplier, quant_func=quant_func, error_func=error_func)


@torch.no_grad()
def _mse_calibrate_weights(model, name_to_module, step_size, start_multiplier, stop_multiplier, fp8_scale_sweep):
    """MSE-refine every eligible weight quantizer in place (reference :779-826)."""
    seen = set()
    for parent in name_to_module.values():
        if id(parent) in seen or not isinstance(parent, QuantModule):
            continue
        seen.add(id(parent))
        for weight, weight_quantizer in parent.iter_weights_for_calibration():
            cal = _make_weight_mse_calibrator(weight_quantizer, step_size, start_multiplier, stop_multiplier,
                                              fp8_scale_sweep)
            if cal is None:
                continue
            weight_quantizer._calibrator = cal
            _run_and_load_max_stats(weight_quantizer, lambda q, w=weight: q(w))
            if hasattr(cal, "reset"):
                cal.reset()


def mse_calibrate(model: nn.Module, forward_loop: ForwardLoop | None = None, distributed_sync=True,
                  step_size: float = 0.1, start_multiplier: float = 0.25, stop_multiplier: float = 4.0,
                  fp8_scale_sweep: bool = False, shared_states=None):
    """Max calibration, then an MSE search of every weight amax (reference :733-776)."""
    max_calibrate(model, forward_loop, distributed_sync, shared_states=shared_states)
    _mse_calibrate_weights(model, dict(model.named_modules()), step_size, start_multiplier, stop_multiplier,
                           fp8_scale_sweep)

_ = math
