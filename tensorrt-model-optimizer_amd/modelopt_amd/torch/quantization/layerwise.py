"""Layer-by-layer calibration (reference: model_calib.py:2051-2189, utils/layerwise_calib.py:104-466).

Same contract as the reference: every decoder layer gets a patched forward driven by a small
per-layer state machine, and the *parent* model forward is re-run for each layer so whatever the
parent builds between layers (rotary tables, masks, caches) is produced naturally:

* ``skip``     -- layers already calibrated return meta-device zeros of their recorded output
                  structure (no compute, no HBM traffic);
* ``run``      -- the layer calibrated last replays its own captured inputs, so its real output
                  feeds the next layer regardless of the meta placeholders upstream;
* ``capture``  -- the target layer records ``(args, kwargs)`` and stops the forward early;
* ``original`` -- untouched.

With ``get_qdq_activations_from_prev_layer=False`` (max / awq default) the next layer's inputs are
captured with the current layer's quantizers disabled, so the amax values equal a whole-model
calibration's.  One layer's activations are resident at a time, which is what makes a 70B model's
calibration fit next to its weights; on MI355X (288 GB) that is a choice, not a necessity.

Per-layer checkpoint/resume (``checkpoint_dir``) is implemented as in the reference's
``_CheckpointState``: after each layer the layer's quantizer state (and, when the algorithm mutates
weights, its parameters) plus the next layer's captured inputs are saved; a restart resumes from
the first layer without a completion marker.
"""

from __future__ import annotations

import json
import os
from collections import deque
from dataclasses import dataclass, field
from typing import Any, Callable

import torch
import torch.nn as nn

from .conversion import set_quantizer_by_cfg_context
from .nn import SequentialQuantizer, TensorQuantizer

__all__ = ["LayerActivationCollector", "layerwise_calibrate"]


class _EarlyStopForwardError(Exception):
    """Raised by a capturing layer to end the parent forward."""


@dataclass
class _LayerCalibState:
    mode: str = "original"
    name: str = ""
    cached_inputs: deque = field(default_factory=deque)
    collected_inputs: list = field(default_factory=list)
    output_meta: Any = None


def _output_meta(out):
    if isinstance(out, torch.Tensor):
        return ("tensor", out.shape, out.dtype)
    if isinstance(out, tuple):
        return ("tuple", tuple(_output_meta(o) for o in out))
    if isinstance(out, list):
        return ("list", [_output_meta(o) for o in out])
    return ("other", out)


def _zeros_from_meta(meta):
    tag = meta[0]
    if tag == "tensor":
        return torch.zeros(meta[1], dtype=meta[2], device="meta")
    if tag == "tuple":
        return tuple(_zeros_from_meta(m) for m in meta[1])
    if tag == "list":
        return [_zeros_from_meta(m) for m in meta[1]]
    return meta[1]


class LayerActivationCollector:
    """Skip / run / capture patching of a model's decoder layers (layerwise_calib.py:104)."""

    _decoder_layer_support: list = []
    _ATTR = "_layerwise_calib"

    def __init__(self, model: nn.Module):
        self.model = model
        self._layers: nn.ModuleList | None = None
        self._idx: dict[nn.Module, int] = {}
        self._patched = False

    @classmethod
    def register_decoder_layer_support(cls, is_supported: Callable, discoverer: Callable):
        entry = (is_supported, discoverer)
        if entry not in cls._decoder_layer_support:
            cls._decoder_layer_support.append(entry)

    @staticmethod
    def get_decoder_layers(model: nn.Module):
        for is_supported, discoverer in LayerActivationCollector._decoder_layer_support:
            if is_supported(model):
                layers = discoverer(model)
                if layers is not None:
                    return layers
        return None

    @staticmethod
    def is_supported(model: nn.Module) -> bool:
        return LayerActivationCollector.get_decoder_layers(model) is not None

    # -- patching --------------------------------------------------------------------------
    def patch(self, layers: nn.ModuleList | None = None):
        self._layers = layers if layers is not None else self.get_decoder_layers(self.model)
        assert self._layers is not None, "no decoder layers found"
        names = {m: n for n, m in self.model.named_modules()}
        self._idx = {layer: i for i, layer in enumerate(self._layers)}

        def layer_forward(mod, *args, **kwargs):
            st: _LayerCalibState = mod.__dict__[LayerActivationCollector._ATTR]
            if st.mode == "skip":
                if st.output_meta is None:
                    raise RuntimeError(f"layer {st.name} is in 'skip' mode without output metadata")
                return _zeros_from_meta(st.output_meta)
            if st.mode == "run":
                assert st.cached_inputs, f"layer {st.name} has no cached inputs to replay"
                a, k = st.cached_inputs.popleft()
                out = mod.__dict__["_lw_original_forward"](*a, **_fresh_kwargs(k))
                st.output_meta = _output_meta(out)
                return out
            if st.mode == "capture":
                st.collected_inputs.append((args, kwargs))
                raise _EarlyStopForwardError()
            return mod.__dict__["_lw_original_forward"](*args, **kwargs)

        def model_forward(mod, *args, **kwargs):
            try:
                return mod.__dict__["_lw_original_forward"](*args, **kwargs)
            except _EarlyStopForwardError:
                return None
            except RuntimeError as e:
                if "meta" in str(e).lower():
                    raise RuntimeError(
                        "layerwise calibration feeds skipped decoder layers' outputs as meta "
                        "placeholders; this model runs real-device ops on the hidden state between "
                        "decoder layers -- use whole-model calibration for it"
                    ) from e
                raise

        self._saved = {}
        for m, fwd in [*((layer, layer_forward) for layer in self._layers), (self.model, model_forward)]:
            self._saved[id(m)] = m.__dict__.get("forward")  # an instance-level forward, if any
            m.__dict__["_lw_original_forward"] = m.forward
            m.forward = fwd.__get__(m)
        for layer in self._layers:
            layer.__dict__[self._ATTR] = _LayerCalibState(name=names.get(layer, type(layer).__name__))
        self._patched = True

    def unpatch(self):
        if not self._patched:
            return
        for m in [*(self._layers or []), self.model]:
            for k in ("forward", "_lw_original_forward", self._ATTR):
                m.__dict__.pop(k, None)
            if self._saved.get(id(m)) is not None:
                m.__dict__["forward"] = self._saved[id(m)]
        self._patched = False

    # -- state machine ---------------------------------------------------------------------
    def _state(self, i) -> _LayerCalibState:
        return self._layers[i].__dict__[self._ATTR]

    def _set_layer_states(self, i: int):
        """Layer i-2 -> skip, layer i-1 -> run (replay), layer i -> capture."""
        if i > 1:
            s = self._state(i - 2)
            s.mode = "skip"
            s.cached_inputs.clear()
        if i > 0:
            prev = self._state(i - 1)
            if prev.mode != "skip":
                if not prev.collected_inputs:
                    raise RuntimeError(f"layer {i - 1} ({prev.name}) has no collected inputs to replay")
                prev.mode = "run"
                prev.cached_inputs = deque(prev.collected_inputs)
                prev.collected_inputs = []
        cur = self._state(i)
        cur.mode = "capture"
        cur.collected_inputs = []

    @torch.no_grad()
    def get_input_activations(self, layer: nn.Module, forward_loop: Callable) -> list:
        if not self._patched:
            raise RuntimeError("get_input_activations() requires patch() first")
        i = self._idx[layer]
        self._set_layer_states(i)
        st = self._state(i)
        try:
            forward_loop(self.model)
        except Exception:
            st.mode = "original"
            st.collected_inputs = []
            raise
        if not st.collected_inputs:
            st.mode = "original"
            raise RuntimeError(f"layer {st.name!r} collected no inputs during forward_loop")
        inputs = list(st.collected_inputs)
        st.mode = "original"
        return inputs

    def cache_outputs_for_next_layer_calib(self, layer: nn.Module, forward_loop: Callable) -> list:
        i = self._idx[layer]
        assert i + 1 < len(self._layers), "no next layer"
        return self.get_input_activations(self._layers[i + 1], forward_loop)

    def seed_resumed(self, start: int, inputs: list, output_metas: list):
        """Resume at layer `start`: earlier layers skip with their recorded output metadata."""
        for i in range(start):
            s = self._state(i)
            s.mode = "skip"
            s.output_meta = output_metas[i]
        s = self._state(start)
        s.collected_inputs = inputs
        s.mode = "original"


# ---- checkpoint / resume --------------------------------------------------------------------
class _CheckpointState:
    """Per-layer checkpoints under ``checkpoint_dir`` (reference model_calib.py _CheckpointState)."""

    def __init__(self, root: str, num_layers: int, save_every: int, calib_mutates_weights: bool):
        self.root, self.n, self.save_every, self.mut = root, num_layers, save_every, calib_mutates_weights
        os.makedirs(root, exist_ok=True)
        meta = os.path.join(root, "progress.json")
        self.done = json.load(open(meta))["completed"] if os.path.exists(meta) else -1
        # resume needs the next-inputs cache of the last completed (flushed) layer
        while self.done >= 0 and not os.path.exists(self._inputs_path(self.done)):
            self.done -= 1

    @property
    def start_layer(self) -> int:
        return self.done + 1

    def _layer_path(self, i):
        return os.path.join(self.root, f"layer_{i:04d}.pt")

    def _inputs_path(self, i):
        return os.path.join(self.root, f"next_inputs_{i:04d}.pt")

    @staticmethod
    def _layer_state(layer: nn.Module, with_weights: bool) -> dict:
        q = {n: m.state_dict() for n, m in layer.named_modules() if isinstance(m, (TensorQuantizer, SequentialQuantizer))}
        d = {"quantizers": q, "output_meta": layer.__dict__[LayerActivationCollector._ATTR].output_meta}
        if with_weights:
            d["params"] = {k: v.detach().cpu() for k, v in layer.state_dict().items() if "quantizer" not in k}
        return d

    def save(self, i: int, layer: nn.Module, next_inputs: list | None):
        torch.save(self._layer_state(layer, self.mut), self._layer_path(i))
        last = i + 1 >= self.n
        if last or (i + 1) % self.save_every == 0:
            if next_inputs is not None:
                torch.save(_to_cpu(next_inputs), self._inputs_path(i))
            with open(os.path.join(self.root, "progress.json"), "w") as f:
                json.dump({"completed": i, "num_layers": self.n}, f)
            for j in range(i):  # older activation caches are no longer needed
                p = self._inputs_path(j)
                if os.path.exists(p):
                    os.remove(p)

    def restore_layers(self, layers: nn.ModuleList, upto: int):
        metas = []
        for i in range(upto):
            # our own files: tensors + plain metadata (torch.Size / dtype / None)
            d = torch.load(self._layer_path(i), map_location="cpu", weights_only=False)
            layer = layers[i]
            dev = next((p.device for p in layer.parameters()), torch.device("cpu"))
            if "params" in d:
                sd = {k: v.to(dev) for k, v in d["params"].items()}
                layer.load_state_dict(sd, strict=False)
            mods = dict(layer.named_modules())
            for n, sd in d["quantizers"].items():
                q = mods.get(n)
                if isinstance(q, TensorQuantizer):
                    if "_amax" in sd:
                        q.amax = sd["_amax"].to(dev)
                    if "_pre_quant_scale" in sd:
                        q.pre_quant_scale = sd["_pre_quant_scale"].to(dev)
            metas.append(d["output_meta"])
        return metas

    def load_inputs(self, i: int, device) -> list:
        return _to_device(torch.load(self._inputs_path(i), map_location="cpu", weights_only=False), device)


def _to_cpu(obj):
    return _map_tensors(obj, lambda t: t.detach().cpu())


def _to_device(obj, device):
    return _map_tensors(obj, lambda t: t.to(device))


def _map_tensors(obj, fn):
    if isinstance(obj, torch.Tensor):
        return fn(obj)
    if isinstance(obj, tuple):
        return tuple(_map_tensors(o, fn) for o in obj)
    if isinstance(obj, list):
        return [_map_tensors(o, fn) for o in obj]
    if isinstance(obj, dict):
        return {k: _map_tensors(v, fn) for k, v in obj.items()}
    return obj


def _fresh_kwargs(k: dict) -> dict:
    """A replayed layer must start from an empty KV cache: drop the captured cache object (its
    contents depend on which replays already ran; transformers-5 ``DynamicCache.reset`` zeroes
    but keeps the cached length, which would corrupt the attention)."""
    if k.get("past_key_values") is not None:
        k = dict(k)
        k["past_key_values"] = None
    return k


def _strip_cache(inputs: list) -> list:
    return [(a, _fresh_kwargs(k)) for a, k in inputs]


@torch.no_grad()
def layerwise_calibrate(
    model: nn.Module,
    forward_loop: Callable,
    calib_func: Callable,
    checkpoint_dir: str | None = None,
    get_qdq_activations_from_prev_layer: bool = False,
    save_every: int = 1,
    calib_mutates_weights: bool = True,
    **calib_kwargs,
):
    """Apply ``calib_func(layer, layer_forward_loop, **calib_kwargs)`` one decoder layer at a time."""
    if forward_loop is None:
        raise ValueError("forward_loop must not be None for layerwise calibration.")
    layers = LayerActivationCollector.get_decoder_layers(model)
    if layers is None or len(layers) == 0:
        raise ValueError("Could not find transformer layers in model; layerwise calibration needs them.")
    n = len(layers)
    ckpt = _CheckpointState(checkpoint_dir, n, save_every, calib_mutates_weights) if checkpoint_dir else None
    start = ckpt.start_layer if ckpt else 0
    if start >= n:
        ckpt.restore_layers(layers, n)
        return

    collector = LayerActivationCollector(model)
    try:
        collector.patch(layers)
        if start > 0:
            metas = ckpt.restore_layers(layers, start)
            dev = next((p.device for p in layers[start].parameters()), torch.device("cpu"))
            inputs = ckpt.load_inputs(start - 1, dev)
            collector.seed_resumed(start, inputs, metas)
        else:
            inputs = collector.get_input_activations(layers[0], forward_loop)

        for i in range(start, n):
            layer = layers[i]
            cur = inputs

            def layer_loop(m, _inputs=cur):
                for a, k in _strip_cache(_inputs):
                    m(*a, **k)

            last = i + 1 >= n
            next_inputs = None
            if not last and not get_qdq_activations_from_prev_layer:
                with set_quantizer_by_cfg_context(layer, [{"quantizer_name": "*", "enable": False}]):
                    next_inputs = collector.cache_outputs_for_next_layer_calib(layer, forward_loop)
                # the capture left this layer in 'run' mode with an empty replay queue
                collector._state(i).mode = "original"
            calib_func(layer, layer_loop, **calib_kwargs)
            if not last and get_qdq_activations_from_prev_layer:
                next_inputs = collector.cache_outputs_for_next_layer_calib(layer, forward_loop)
            if ckpt:
                ckpt.save(i, layer, next_inputs)
            inputs = next_inputs
    finally:
        collector.unpatch()
