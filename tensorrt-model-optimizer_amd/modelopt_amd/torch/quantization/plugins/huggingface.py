"""HuggingFace MoE plugins on the PTQ hot path (reference: plugins/huggingface.py).

``_QuantFusedExperts`` (reference :976-1115) wraps transformers-5 fused expert containers
(``gate_up_proj`` [E, 2I, H] + ``down_proj`` [E, H, I] 3-D parameters; Mixtral, Qwen-MoE, OLMoE,
...): one shared input quantizer per projection and one weight quantizer per expert, applied by
intercepting the two ``F.linear`` calls the HF eager expert loop makes per expert (the expert index
is recovered from the weight slice's storage offset).  Registered on the fly for every module type
with that structure (reference :1697-1720), so ``mtq.quantize`` on a Mixtral model needs no setup.
"""

from __future__ import annotations

import contextlib
import functools
import inspect

import torch
import torch.nn as nn

from ..nn.modules import quant_linear as _quant_linear
from ..nn.modules.quant_module import QuantModule, QuantModuleRegistry
from ..nn.modules.tensor_quantizer import TensorQuantizer
from . import register_on_the_fly

__all__ = [
    "_QuantAttention",
    "_QuantFusedExperts",
    "force_eager_experts_impl_on_the_fly",
    "register_fused_experts_on_the_fly",
    "register_hf_attentions_on_the_fly",
]


@contextlib.contextmanager
def _replace_function(package, name, new_fn):
    old = getattr(package, name)
    setattr(package, name, new_fn)
    try:
        yield
    finally:
        setattr(package, name, old)


class _QuantFusedExperts(QuantModule):
    _first_proj_attr = "gate_up_proj"

    def _setup(self):
        n = self.num_experts
        setattr(self, f"{self._first_proj_attr}_input_quantizer", TensorQuantizer())
        setattr(self, f"{self._first_proj_attr}_weight_quantizers", nn.ModuleList([TensorQuantizer() for _ in range(n)]))
        self.down_proj_input_quantizer = TensorQuantizer()
        self.down_proj_weight_quantizers = nn.ModuleList([TensorQuantizer() for _ in range(n)])
        self.__dict__["_down_proj_linear"] = False
        self.__dict__["_current_expert_idx"] = 0

    def _get_expert_idx_from_first_proj(self, weight: torch.Tensor) -> int:
        first = getattr(self, self._first_proj_attr)
        stride = first.stride(0)
        if stride == 0:
            return 0
        idx = (weight.storage_offset() - first.storage_offset()) // stride
        assert 0 <= idx < self.num_experts, (
            f"Computed expert index {idx} out of range [0, {self.num_experts}). "
            "This can happen if the weight was .contiguous()-copied or redistributed."
        )
        return idx

    def forward(self, *args, **kwargs):
        orig_linear = torch.nn.functional.linear
        first_in = getattr(self, f"{self._first_proj_attr}_input_quantizer")
        first_w = getattr(self, f"{self._first_proj_attr}_weight_quantizers")
        d = self.__dict__
        d["_first_in_done"] = False
        # The first projection's input of expert e is hidden_states[token_idx_e]: when every token
        # is routed to some expert and the shared input quantizer acts on each token on its own,
        # applying it ONCE to hidden_states (collect and/or fake quant) equals applying it to each
        # expert's gather -- max over the union = max of the per-expert maxima, and a per-element
        # qdq commutes with the gather -- so one reduction / qdq launch replaces E of them.  Rows
        # routed to no local expert (index outside [0, E): expert-parallel sentinels) are zeroed
        # first, on the device (no host sync): |0| adds nothing to a running max, and no expert
        # gathers those rows.
        args = list(args)
        hs = args[0] if args else kwargs.get("hidden_states")
        idx_t = args[1] if len(args) > 1 else kwargs.get("top_k_index")
        if (
            isinstance(hs, torch.Tensor) and hs.dim() == 2 and isinstance(idx_t, torch.Tensor)
            and idx_t.dim() == 2 and idx_t.shape[0] == hs.shape[0] and _token_separable(first_in)
        ):
            if hs.is_cuda and idx_t.dtype == torch.int64 and idx_t.device == hs.device:
                # one library pass (no compare / any / where kernels to load on first use)
                from modelopt_amd._ext import ops as _ops

                masked = first_in(_ops().mask_unrouted_rows(hs, idx_t, self.num_experts))
            else:
                routed = ((idx_t >= 0) & (idx_t < self.num_experts)).any(dim=-1, keepdim=True)
                masked = first_in(torch.where(routed, hs, hs.new_zeros(())))
            if not first_in.returns_input_unchanged():
                # fake quant: the experts read the quantised tokens (a collect-only call hands
                # back the masked copy itself: the experts read hs, whose unrouted rows no
                # expert gathers)
                if args:
                    args[0] = masked
                else:
                    kwargs["hidden_states"] = masked
            d["_first_in_done"] = True
        # The eager expert loop syncs the host once per expert (torch.where, and the expert-index
        # slice of the fused weight), so host time between such a sync and the next GEMM launch
        # is GPU idle time.  Quantizers that hand their input back unchanged (calibration collect,
        # no fake quant) are therefore called AFTER the GEMM is launched -- the same calls on the
        # same tensors, their host time behind the GEMM -- and whether they do is decided once
        # per forward here, not per expert.
        first_late = d["_first_in_done"] and all(_returns_input_q(q) for q in first_w)
        down_late = _returns_input_q(self.down_proj_input_quantizer) and all(
            _returns_input_q(q) for q in self.down_proj_weight_quantizers)

        def _quantized_linear(input, weight, bias=None):
            if d["_down_proj_linear"]:
                d["_down_proj_linear"] = False
                idx = d["_current_expert_idx"]
                wq = self.down_proj_weight_quantizers[idx]
                if down_late and type(input) is torch.Tensor and type(weight) is torch.Tensor:
                    out = orig_linear(input, weight, bias)
                    self.down_proj_input_quantizer(input)
                    if not _collected_already(wq, weight):
                        wq(weight)
                    return out
                input = self.down_proj_input_quantizer(input)
                if not _collected_already(wq, weight):
                    weight = wq(weight)
                return orig_linear(input, weight, bias)
            d["_down_proj_linear"] = True
            if first_late and type(input) is torch.Tensor and type(weight) is torch.Tensor:
                out = orig_linear(input, weight, bias)
                idx = self._get_expert_idx_from_first_proj(weight)
                d["_current_expert_idx"] = idx
                wq = first_w[idx]
                if not _collected_already(wq, weight):
                    wq(weight)
                return out
            idx = self._get_expert_idx_from_first_proj(weight)
            d["_current_expert_idx"] = idx
            if not d["_first_in_done"]:
                input = first_in(input)
            wq = first_w[idx]
            if not _collected_already(wq, weight):
                weight = wq(weight)
            return orig_linear(input, weight, bias)

        d["_down_proj_linear"] = False
        with _replace_function(torch.nn.functional, "linear", _quantized_linear):
            return self._original_cls.forward(self, *args, **kwargs)

    def iter_weights_for_calibration(self):
        for wname, qname in ((self._first_proj_attr, f"{self._first_proj_attr}_weight_quantizers"),
                             ("down_proj", "down_proj_weight_quantizers")):
            weight = getattr(self, wname, None)
            qs = getattr(self, qname, None)
            if weight is None or qs is None:
                continue
            for idx, q in enumerate(qs):
                yield weight[idx], q

    def fold_weight(self, keep_attrs: bool = False):
        for w, q in self.iter_weights_for_calibration():
            if isinstance(q, TensorQuantizer) and q.fake_quant:
                self._fold_weight_quantizer(q, (w,), keep_attrs)


def _collected_already(q, weight) -> bool:
    """The expert weight quantizer call is a no-op (``calib.max.quantizer_call_is_noop``): a max
    calibration pass whose calibrator has just collected this very expert slice (max_calibrate's
    weight pass collects every slice before the forward loop).  Saves the module call per expert
    and batch of the eager expert loop, whose per-expert host syncs expose every host microsecond."""
    from ..calib.max import quantizer_call_is_noop

    return type(q) is TensorQuantizer and quantizer_call_is_noop(q, weight)


def _returns_input_q(q) -> bool:
    """The TensorQuantizer ``q`` hands a plain tensor input back unchanged (collect-only
    calibration or disabled, no pre_quant_scale, no block reshape; see
    TensorQuantizer.returns_input_unchanged)."""
    return isinstance(q, TensorQuantizer) and q.returns_input_unchanged()


def _token_separable(q) -> bool:
    """Whether ``q`` treats every row (token) of a [tokens, H] input on its own, so that applying
    it to all tokens at once equals applying it to any cover of the tokens by row subsets: disabled;
    or collecting into a MaxCalibrator per tensor / per last-dim channel; and quantizing with a
    static per-tensor / per-last-dim amax or dynamic blocks along the last dim only (MX, NVFP4
    with a static global amax, per-token FP8).  Anything else (NVFP4 whose global amax is taken
    from the call's input, dynamic per-tensor amax, static row blocks, histograms, custom
    backends) keeps the per-expert calls."""
    from ..calib.max import MaxCalibrator

    if type(q) is not TensorQuantizer:
        return False
    if q._disabled:
        return True
    if getattr(q, "backend", None) is not None:
        return False
    last_axis = q.axis is None or q.axis in (-1, 1, (-1,), (1,), [-1], [1])
    if q._if_calib and not q._dynamic:
        if type(q._calibrator) is not MaxCalibrator or not last_axis:
            return False
    if q._if_quant:
        bs = q.block_sizes
        if bs:
            dims = [k for k in bs if isinstance(k, int)]
            if bs.get("type") != "dynamic" or any(k not in (-1, 1) for k in dims):
                return False
            # NVFP4's second-level (per-tensor) scale comes from the global amax: without a static
            # one it is the amax of whatever tensor the call sees (_get_amax -> reduce_amax), so
            # all routed tokens at once would differ from each expert's token gather
            if bs.get("scale_bits") == (4, 3) and getattr(q, "_amax", None) is None:
                return False
        elif q._dynamic or not last_axis:
            return False
    return True


def _has_num_experts(obj) -> bool:
    return hasattr(obj, "num_experts") or hasattr(obj, "n_routed_experts")


def _num_experts(*objs) -> int:
    for obj in objs:
        for attr in ("num_experts", "n_routed_experts"):
            n = getattr(obj, attr, None) if obj is not None else None
            if n:
                return int(n)
    return 0


class _QuantSparseSequentialMoe(QuantModule):
    """MoE block whose ``experts`` is iterable (one module per expert, each expert's linears are
    QuantLinear on their own) -- reference plugins/huggingface.py:623-750.

    With ``_moe_calib_experts_ratio`` set (``algorithm={"moe_calib_experts_ratio": r}``), every
    calibration forward first routes the tokens to ``max(top_k, round(E * r))`` experts (output
    discarded, so more experts see tokens and get activation amax), then runs the original
    ``top_k`` forward; tokens routed per expert are counted in ``expert_token_count`` while
    ``r < 1``.  Without it the forward is the original one."""

    def _setup(self):
        self._moe_calib_experts_ratio = None
        self._token_counting_initialized = False
        self._count_expert_tokens = False

    def _init_token_counting(self):
        self._token_counting_initialized = True
        n = _num_experts(getattr(self, "gate", None), self, getattr(self, "experts", None))
        if n == 0:
            import warnings

            warnings.warn(f"{type(self).__name__}: could not resolve num_experts; expert routing is not tracked.")
            return
        dev = next(self.parameters()).device
        self.register_buffer("expert_token_count", torch.zeros(n, dtype=torch.long, device=dev), persistent=False)
        if hasattr(self, "gate"):
            self.gate.register_forward_hook(self._gate_forward_hook)

    def _gate_forward_hook(self, module, input, output):
        if not self._count_expert_tokens or not hasattr(self, "expert_token_count"):
            return
        with torch.no_grad():
            if isinstance(output, tuple) and len(output) >= 3:  # transformers-5 TopKRouter
                indices = output[2]
            else:
                logits = output[0] if isinstance(output, tuple) else output
                top_k = self.gate.top_k if hasattr(self.gate, "top_k") else self.top_k
                indices = torch.topk(logits.float(), top_k, dim=-1)[1]
            counts = torch.bincount(indices.reshape(-1), minlength=self.expert_token_count.shape[0])
            self.expert_token_count += counts.to(self.expert_token_count.device)

    def _top_k_owner(self):
        if hasattr(self, "gate") and hasattr(self.gate, "top_k"):
            return self.gate
        return self

    def forward(self, hidden_states, *args, **kwargs):
        fwd = self._original_cls.forward
        if self._moe_calib_experts_ratio is None:
            return fwd(self, hidden_states, *args, **kwargs)
        is_calib = any(getattr(m, "_if_calib", False) for m in self.experts.modules())
        if is_calib:
            self._count_expert_tokens = self._moe_calib_experts_ratio < 1.0
            if self._count_expert_tokens and not self._token_counting_initialized:
                self._init_token_counting()
            owner = self._top_k_owner()
            n = _num_experts(getattr(self, "gate", None), self) or len(self.experts)
            original = owner.top_k
            owner.top_k = max(original, round(n * self._moe_calib_experts_ratio))
            try:
                fwd(self, hidden_states, *args, **kwargs)
            finally:
                owner.top_k = original
            self._count_expert_tokens = False
        out = fwd(self, hidden_states, *args, **kwargs)
        self._count_expert_tokens = False
        return out

    def layer_sync_moe_local_experts_amax(self, sync_weight_amax=False):
        """Element-wise max of every expert's input (and optionally weight) amax, written back
        to all experts; experts that saw no token get a weight-only max calibration (reference
        core_utils.py:710-750).  Skipped with ``_moe_calib_experts_ratio`` set."""
        if self._moe_calib_experts_ratio is not None:
            return
        from ..model_calib import max_calibrate

        amax: dict = {}
        for expert in self.experts:
            for name, m in expert.named_modules():
                if not isinstance(m, TensorQuantizer) or m.amax is None:
                    continue
                if "input_quantizer" in name or (sync_weight_amax and "weight_quantizer" in name):
                    a = m.amax.detach().clone()
                    amax[name] = a if name not in amax else torch.maximum(amax[name], a)
        for expert in self.experts:
            for name, m in expert.named_modules():
                if isinstance(m, TensorQuantizer) and name in amax:
                    m.amax = amax[name].detach().clone()
        for expert in self.experts:
            for name, m in expert.named_modules():
                if name.endswith("weight_quantizer") and m.is_enabled and m.amax is None:
                    w = expert.state_dict().get(name.replace("weight_quantizer", "weight"))
                    if w is not None:
                        max_calibrate(m, lambda q, w=w: q(w), distributed_sync=False)


def _is_sparse_sequential_moe_block(module) -> bool:
    """``gate`` (top_k + num_experts) + iterable ``experts`` (reference :1592-1622)."""
    if not hasattr(module, "experts") or not hasattr(module.experts, "__iter__"):
        return False
    gate = getattr(module, "gate", None)
    if gate is not None and hasattr(gate, "top_k") and _has_num_experts(gate):
        return True
    if hasattr(module, "top_k"):
        if not _has_num_experts(module) and hasattr(module.experts, "__len__"):
            module.num_experts = len(module.experts)
        return _has_num_experts(module)
    return False


@register_on_the_fly
def register_sparse_moe_on_the_fly(model):
    """Register every sparse sequential MoE block type of ``model`` (reference :1625-1649)."""
    seen = set()
    for _, module in model.named_modules():
        t = type(module)
        if t in seen or t in QuantModuleRegistry:
            continue
        seen.add(t)
        if _is_sparse_sequential_moe_block(module):
            QuantModuleRegistry.register({t: f"hf.{t.__name__}"})(_QuantSparseSequentialMoe)


def _is_fused_experts_module(module) -> bool:
    return _fused_experts_wrapper_class(module) is not None


def _fused_experts_wrapper_class(module):
    if not hasattr(module, "num_experts"):
        return None
    down = getattr(module, "down_proj", None)
    if not isinstance(down, torch.Tensor) or down.dim() != 3:
        return None
    gate_up = getattr(module, "gate_up_proj", None)
    if isinstance(gate_up, torch.Tensor) and gate_up.dim() == 3:
        return _QuantFusedExperts
    return None


@register_on_the_fly
def register_fused_experts_on_the_fly(model):
    """Register every fused-experts module type found in ``model`` (reference :1697-1720)."""
    seen = set()
    for _, module in model.named_modules():
        t = type(module)
        if t in seen or t in QuantModuleRegistry:
            continue
        seen.add(t)
        cls = _fused_experts_wrapper_class(module)
        if cls is not None:
            QuantModuleRegistry.register({t: f"hf.{t.__name__}"})(cls)


@register_on_the_fly
def force_eager_experts_impl_on_the_fly(model):
    """Pin HF fused experts to the eager ``F.linear`` loop (reference :1725-1753).

    transformers >= 5 dispatches ``@use_experts_implementation`` forwards on
    ``config._experts_implementation`` (``grouped_mm`` / ``batched_mm`` on GPU), which never calls
    ``F.linear`` and would silently bypass the expert quantizers.
    """
    if not any(_is_fused_experts_module(m) for m in model.modules()):
        return

    def _force(cfg):
        if cfg is None:
            return
        if hasattr(cfg, "_experts_implementation"):
            cfg._experts_implementation = "eager"
        for sub in ("text_config", "vision_config", "audio_config", "speech_config"):
            if hasattr(cfg, sub):
                _force(getattr(cfg, sub))

    _force(getattr(model, "config", None))


_ATTN_MODULES: dict = {}


def _attn_module_of(cls):
    """``inspect.getmodule`` of an attention class, memoised (called on every attention forward)."""
    mod = _ATTN_MODULES.get(cls)
    if mod is None:
        mod = _ATTN_MODULES[cls] = inspect.getmodule(cls)
    return mod


class _QuantAttention(QuantModule):
    """KV-cache / attention-BMM quantization for transformers attention modules that dispatch
    through ``ALL_ATTENTION_FUNCTIONS`` (reference plugins/huggingface.py:78-410).

    ``q/k/v_bmm_quantizer`` fake-quantise the query / key / value states handed to the attention
    function (after RoPE and the KV-cache update, as the reference); they are per-tensor HIP
    passes that read the transposed ``[B, H, S, D]`` states in place (no ``.contiguous()`` copy).
    ``p_bmm_quantizer`` fake-quantises the softmax probabilities as the reference dispatches it
    (:125-251): per-tensor FP8 or dynamic NVFP4 block 16 on causal attention run the fused MFMA
    flash attention with the P qdq inside (``mtq_attention_fwd``, csrc/mtq_attention.hip; the
    reference's Triton ``_attn_fwd``), non-causal attention wraps ``F.softmax`` of the original
    attention function, and any other P format leaves the attention unquantised (the reference
    hands those to the optional ``kitchen`` package, which is not part of this path)."""

    def _setup(self):
        self.q_bmm_quantizer = TensorQuantizer()
        self.k_bmm_quantizer = TensorQuantizer()
        self.v_bmm_quantizer = TensorQuantizer()
        self.p_bmm_quantizer = TensorQuantizer()

    @staticmethod
    def get_attn_type(attn_module) -> type:
        return getattr(attn_module, "_original_cls", type(attn_module))

    @staticmethod
    def is_compatible_attention(attn_cls) -> bool:
        mod = inspect.getmodule(attn_cls)
        return getattr(mod, "ALL_ATTENTION_FUNCTIONS", None) is not None

    def _p_qdq_mode(self) -> str | None:
        """reference :125-143: "fp8" (per-tensor E4M3), "nvfp4" (dynamic, block 16) or None."""
        pq = self.p_bmm_quantizer
        if not pq.is_enabled:
            return None
        if pq.is_fp8:
            return "fp8"
        if pq.is_nvfp4_dynamic and (pq.block_sizes or {}).get(-1, None) == 16:
            return "nvfp4"
        return None

    def _fused_qdq_attention(self, p_qdq, query_states, key_states, value_states, **kwargs):
        """reference ``_triton_qdq_attention`` :145-195 on the MFMA kernel: the calibrated (or
        user-set) per-tensor amax of ``p_bmm_quantizer`` is the P scale, 1.0 without one."""
        from ...kernels.common.attention import attention_forward, validate_attention_envelope

        attention_mask = kwargs.pop("attention_mask", None)
        validate_attention_envelope(self, query_states, key_states, attention_mask, **kwargs)
        p_qdq_amax = None
        pq_amax = getattr(self.p_bmm_quantizer, "_amax", None)
        if pq_amax is not None:
            if pq_amax.numel() != 1:
                raise NotImplementedError(
                    "p_bmm_quantizer via the Triton attention kernel only supports a "
                    f"per-tensor (scalar) amax, got shape {tuple(pq_amax.shape)}."
                )
            p_qdq_amax = float(pq_amax)
        scaling = kwargs.get("scaling")
        if scaling is None:
            scaling = query_states.shape[-1] ** -0.5
        return attention_forward(self, query_states, key_states, value_states, attention_mask, scaling,
                                 p_qdq=p_qdq, p_qdq_amax=p_qdq_amax)

    def _eager_p_qdq_attention(self, original, query_states, key_states, value_states, **kwargs):
        """reference :197-218: ``F.softmax`` replaced by ``p_bmm_quantizer(softmax(...))`` inside
        the original attention function (an SDPA-fused softmax is unaffected, as there)."""
        pq = self.p_bmm_quantizer
        orig_softmax = torch.nn.functional.softmax

        def _quantized_softmax(*s_args, **s_kwargs):
            return pq(orig_softmax(*s_args, **s_kwargs))

        with _replace_function(torch.nn.functional, "softmax", _quantized_softmax):
            return original(self, query_states, key_states, value_states, **kwargs)

    @staticmethod
    def _quantized_attention(original_attention_interface, self, query_states, key_states,
                             value_states, *args, **kwargs):
        query_states = self.q_bmm_quantizer(query_states)
        key_states = self.k_bmm_quantizer(key_states)
        value_states = self.v_bmm_quantizer(value_states)
        p_qdq = self._p_qdq_mode()
        if p_qdq is not None:
            if args:  # the attention interface passes attention_mask positionally (reference :240-241)
                kwargs["attention_mask"] = args[0]
            if kwargs.get("is_causal") is False or getattr(self, "is_causal", True) is False:
                return self._eager_p_qdq_attention(original_attention_interface, query_states, key_states,
                                                   value_states, **kwargs)
            return self._fused_qdq_attention(p_qdq, query_states, key_states, value_states, **kwargs)
        return original_attention_interface(self, query_states, key_states, value_states, *args, **kwargs)

    def forward(self, *args, **kwargs):
        cfg = getattr(self, "config", None)
        if cfg is None:
            cfg = next((getattr(m, "config", None) for m in self.children() if hasattr(m, "config")), None)
        impl = getattr(cfg, "_attn_implementation", None) if cfg is not None else None
        eager = impl is None or impl == "eager" or (impl == "sdpa" and kwargs.get("output_attentions", False))
        module = _attn_module_of(self.get_attn_type(self))
        eager_fn = getattr(module, "eager_attention_forward", None)
        if eager:
            if eager_fn is None:
                raise AssertionError(
                    f"Module {module} does not have `eager_attention_forward` to enable KV Cache quantization. "
                    "Please use a different attention implementation such as `sdpa`."
                )
            original = eager_fn
        else:
            original = module.ALL_ATTENTION_FUNCTIONS[impl]
        patch_fn = functools.partial(self._quantized_attention, original)
        registry = module.ALL_ATTENTION_FUNCTIONS
        had_local = (not eager) and impl in registry._local_mapping
        if eager:
            module.eager_attention_forward = patch_fn
        else:
            registry[impl] = patch_fn
        # decode-shaped steps: the q/k/v projections (same hidden state) as one fused launch
        projs = self._qkv_projections()
        if projs:
            group = _quant_linear.ProjectionGroup(projs)
            for m in projs:
                m.__dict__["_projection_group"] = group
        try:
            return self._original_cls.forward(self, *args, **kwargs)
        finally:
            for m in projs:
                m.__dict__.pop("_projection_group", None)
            if eager:
                module.eager_attention_forward = original
            elif had_local:
                registry[impl] = original
            else:
                del registry[impl]

    def _qkv_projections(self) -> list:
        """q_proj / k_proj / v_proj when they are separate quantized linears (MI355X addition:
        decode steps run them as one grouped launch, see ``ProjectionGroup``)."""
        if not _quant_linear._FUSED[0]:
            return []
        mods = [self._modules.get(n) for n in ("q_proj", "k_proj", "v_proj")]
        if any(not isinstance(m, _quant_linear._QuantLinear) for m in mods):
            return []
        return mods


def _wraps_nested_attention(module) -> bool:
    return any(type(c).__name__.endswith("Attention") for c in module.children())


@register_on_the_fly
def register_hf_attentions_on_the_fly(model):
    """Register the transformers attention classes of ``model`` for KV-cache / BMM quantization
    (reference :412-460)."""
    if not _is_hf_model(model):
        return
    for _, module in model.named_modules():
        if not type(module).__name__.endswith("Attention") or _wraps_nested_attention(module):
            continue
        t = _QuantAttention.get_attn_type(module)
        if t in QuantModuleRegistry or not _QuantAttention.is_compatible_attention(t):
            continue
        QuantModuleRegistry.register({t: f"hf.{t.__name__}"})(_QuantAttention)
        print(f"Registered {t} to {_QuantAttention.__name__} for KV Cache quantization")


def _is_hf_model(model) -> bool:
    try:
        from transformers import PreTrainedModel
    except ImportError:  # pragma: no cover
        return False
    return isinstance(model, PreTrainedModel)


def get_homogeneous_hf_decoder_layers(model):
    """``model.model[.language_model].layers`` of an HF causal LM (reference :1799-1811)."""
    if not _is_hf_model(model):
        return None
    dec = getattr(model, "model", model)
    dec = getattr(dec, "language_model", dec)
    return getattr(dec, "layers", None)


def _register_layerwise_support():
    from ..layerwise import LayerActivationCollector

    LayerActivationCollector.register_decoder_layer_support(_is_hf_model, get_homogeneous_hf_decoder_layers)


_register_layerwise_support()
