"""Layer-sharded (pipelined) calibration across the GPUs of one node.

The reference reaches multi-GPU calibration through Megatron / FSDP plugins and syncs each
quantizer's amax with its own collective (tensor_quantizer.py:1373-1385).  Here the decoder layers
of an HF causal LM are split into contiguous stages, one per rank (80 Llama-3-70B layers / 8 GPUs
= 10 per GPU); the unchanged user ``forward_loop`` runs on every rank and the decoder-layer
forwards are patched so that

* layers before this rank's stage pass the (embedding) hidden states through untouched -- every
  rank materialises the embedding and rotary tables so the parent forward builds real position
  embeddings / masks, but no decoder compute happens outside the owning rank;
* the stage's first layer replaces its input with the hidden states received from rank r-1
  (``dist.recv`` -> RCCL point-to-point over xGMI);
* the stage's last layer sends its output to rank r+1 with a non-blocking ``isend`` (at most
  one in flight, waited before the next send) and ends the forward early (the last rank runs the
  model's tail normally).

Each rank therefore calibrates exactly its own layers' quantizers on the same activations a
single-GPU run would produce, and consecutive batches overlap across stages (batch i on stage r
while batch i+1 is on stage r-1).  The per-stage amax state is then exchanged with ONE packed
``all_reduce(MAX)`` over the world group (every rank ends up with the complete quantizer state,
as export needs): owners contribute their values, other ranks zeros (amax >= 0).  The same
exchange carries every quantizer's ``_pre_quant_scale`` (AWQ / SmoothQuant, > 0), and the static
block weight quantizers are promoted afterwards on every rank (NVFP4's ``_global_amax`` is derived
from the exchanged amax), so non-owners end with the owners' complete quantizer state.

Inside the context the model's forward returns ``None`` on every rank but the last (the stage
stops the forward after sending its hidden states): a ``forward_loop`` must not read outputs.
With the ``gloo`` backend (CPU rehearsal, or several ranks sharing one GPU) device tensors are
staged through host memory for the point-to-point hand-off and the all-reduce.

Decoder layers must return a tensor (transformers >= 5); models whose parent forward mixes the
hidden state between layers are not supported (same restriction as layerwise calibration).
"""

from __future__ import annotations

import contextlib
from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn as nn

from .layerwise import LayerActivationCollector, _EarlyStopForwardError
from .nn import SequentialQuantizer, TensorQuantizer
from .nn.modules import quant_module as _qm

__all__ = ["LayerShardPlan", "layer_shard_plan", "layer_sharded_calibration", "sync_sharded_amax"]


@dataclass(frozen=True)
class LayerShardPlan:
    rank: int
    world: int
    first: int  # first owned decoder layer
    last: int  # one past the last owned decoder layer
    num_layers: int

    @property
    def owned(self) -> range:
        return range(self.first, self.last)


def layer_shard_plan(num_layers: int, rank: int, world: int) -> LayerShardPlan:
    """Contiguous, balanced stages (the first ``num_layers % world`` ranks take one more)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(num_layers, world)
    first = rank * base + min(rank, extra)
    return LayerShardPlan(rank, world, first, first + base + (1 if rank < extra else 0), num_layers)


def _is_gloo(group) -> bool:
    return dist.get_backend(group) == "gloo"


class _Sender:
    """Non-blocking point-to-point sends (RCCL over xGMI; host-staged under gloo, which has no
    device P2P).  At most one send is in flight: the next one first waits for the previous, so the
    stage starts computing batch i+1 while batch i's hidden states are still on the wire and the
    sent tensor stays alive until its transfer completes."""

    def __init__(self):
        self._work = None
        self._tensor = None

    def send(self, t: torch.Tensor, dst: int, group) -> None:
        if t.device.type != "cpu" and _is_gloo(group):
            t = t.cpu()
        self.wait()
        self._work = dist.isend(t, dst=dst, group=group)
        self._tensor = t

    def wait(self) -> None:
        if self._work is not None:
            self._work.wait()
        self._work = self._tensor = None


def _recv(buf: torch.Tensor, src: int, group) -> None:
    if buf.device.type != "cpu" and _is_gloo(group):
        host = torch.empty(buf.shape, dtype=buf.dtype)
        dist.recv(host, src=src, group=group)
        buf.copy_(host)
    else:
        dist.recv(buf, src=src, group=group)


def _hidden_arg(args, kwargs):
    if args:
        return args[0], lambda h: ((h, *args[1:]), kwargs)
    return kwargs["hidden_states"], lambda h: (args, {**kwargs, "hidden_states": h})


@contextlib.contextmanager
def layer_sharded_calibration(model: nn.Module, plan: LayerShardPlan, group=None):
    """Patch ``model`` for pipelined calibration of ``plan``'s stage (see module docstring).

    Inside the context every QuantModule created or converted defaults to no data-parallel amax
    sync (the stages hold different layers; use :func:`sync_sharded_amax` afterwards).
    """
    layers = LayerActivationCollector.get_decoder_layers(model)
    if layers is None:
        raise ValueError("layer-sharded calibration needs a model with discoverable decoder layers")
    if len(layers) != plan.num_layers:
        raise ValueError(f"plan is for {plan.num_layers} layers, model has {len(layers)}")
    prev_rank = plan.rank - 1 if plan.rank > 0 else None
    next_rank = plan.rank + 1 if plan.rank + 1 < plan.world else None
    if group is not None:
        prev_rank = dist.get_global_rank(group, prev_rank) if prev_rank is not None else None
        next_rank = dist.get_global_rank(group, next_rank) if next_rank is not None else None

    saved = []
    sender = _Sender()

    def patch(m, fn):
        saved.append((m, m.__dict__.get("forward")))
        orig = m.forward
        m.forward = fn(orig).__get__(m)

    def passthrough(orig):
        def f(mod, *args, **kwargs):
            h, _ = _hidden_arg(args, kwargs)
            return h

        return f

    def stage_layer(orig, i):
        def f(mod, *args, **kwargs):
            if i == plan.first and prev_rank is not None:
                h, rebuild = _hidden_arg(args, kwargs)
                buf = torch.empty(h.shape, dtype=h.dtype, device=_device_of(mod, h))
                _recv(buf, prev_rank, group)
                args, kwargs = rebuild(buf)
            out = orig(*args, **kwargs)
            if i == plan.last - 1 and next_rank is not None:
                if not isinstance(out, torch.Tensor):
                    raise TypeError("layer-sharded calibration needs decoder layers that return a tensor")
                sender.send(out.contiguous(), next_rank, group)
                raise _EarlyStopForwardError()
            return out

        return f

    def model_fwd(orig):
        def f(mod, *args, **kwargs):
            try:
                return orig(*args, **kwargs)
            except _EarlyStopForwardError:
                return None

        return f

    prev_default = _qm._DEFAULT_DP_GROUP
    _qm._DEFAULT_DP_GROUP = -1
    try:
        for i, layer in enumerate(layers):
            if i < plan.first:
                patch(layer, passthrough)
            elif i < plan.last:
                patch(layer, lambda o, i=i: stage_layer(o, i))
            # layers past the stage are never reached (early stop), except on the last rank
        patch(model, model_fwd)
        for m in model.modules():
            if isinstance(m, _qm.QuantModule):
                m.parallel_state = _qm.ParallelState(data_parallel_group=-1)
        yield plan
        sender.wait()
    finally:
        _qm._DEFAULT_DP_GROUP = prev_default
        for m, fwd in reversed(saved):
            m.__dict__.pop("forward", None)
            if fwd is not None:
                m.__dict__["forward"] = fwd


def _device_of(mod: nn.Module, like: torch.Tensor) -> torch.device:
    for p in mod.parameters():
        if p.device.type != "meta":
            return p.device
    return like.device


def _leaf_quantizers(model: nn.Module):
    for name, m in model.named_modules():
        if isinstance(m, TensorQuantizer) and not isinstance(m, SequentialQuantizer):
            yield name, m


# per-quantizer tensors the owner's calibration produces and every rank needs (all >= 0, so a
# MAX all-reduce with zeros from the non-owners returns the owner's values exactly)
_SYNCED_ATTRS = ("_amax", "_pre_quant_scale")


@torch.no_grad()
def sync_sharded_amax(model: nn.Module, device=None, group=None) -> int:
    """Give every rank the complete quantizer state after layer-sharded calibration.

    The shapes of the owned (real) ``_amax`` / ``_pre_quant_scale`` buffers are exchanged as small
    host objects; the values travel in ONE packed fp32 ``all_reduce(MAX)`` on ``device`` (RCCL on
    MI355X; host-staged under gloo).  Static block weight quantizers are then promoted on every
    rank.  Returns the number of entries in the packed buffer.

    Requirement: the layers a rank does not own hold their parameters on the meta device (as
    ``layer_sharded_calibration`` runs them).  A stage owner's AWQ / SmoothQuant calibration folds
    ``1 / pre_quant_scale`` into ITS weights; a non-owner with real, unfolded weights would get the
    owner's ``pre_quant_scale`` and amax on top of them, so receiving a ``_pre_quant_scale`` into a
    module with real parameters raises.
    """
    if not (dist.is_available() and dist.is_initialized()):
        return 0
    from .model_calib import promote_static_block_weight_quantizers

    mods = dict(_leaf_quantizers(model))
    mine = {}
    for name, q in mods.items():
        for attr in _SYNCED_ATTRS:
            a = q.__dict__.get("_buffers", {}).get(attr, getattr(q, attr, None))
            if isinstance(a, torch.Tensor) and a.device.type != "meta":
                mine[(name, attr)] = (tuple(a.shape), str(a.dtype).replace("torch.", ""))
    world = dist.get_world_size(group)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine, group=group)
    layout = {}
    for d in gathered:
        for k, v in d.items():
            if k in layout and layout[k] != v:
                raise RuntimeError(f"{k[1]} shape/dtype of {k[0]} differs across ranks: {layout[k]} vs {v}")
            layout[k] = v
    keys = sorted(layout)
    sizes = [int(torch.Size(layout[k][0]).numel()) for k in keys]
    total = sum(sizes)
    if device is None:
        device = next((getattr(mods[n], a).device for (n, a) in mine), None)
        device = device or torch.device("cuda", torch.cuda.current_device())
    flat = torch.zeros(total, dtype=torch.float32, device=device)
    off = 0
    for k, sz in zip(keys, sizes):
        if k in mine:
            flat[off : off + sz] = getattr(mods[k[0]], k[1]).detach().reshape(-1).to(device=device, dtype=torch.float32)
        off += sz
    if _is_gloo(group) and flat.device.type != "cpu":
        c = flat.cpu()
        dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
        flat = c.to(device)
    else:
        dist.all_reduce(flat, op=dist.ReduceOp.MAX, group=group)
    named = dict(model.named_modules())
    for name, attr in keys:
        if attr != "_pre_quant_scale" or (name, attr) in mine or name not in mods:
            continue
        parent = named.get(name.rsplit(".", 1)[0]) if "." in name else model
        if parent is not None and any(p.device.type != "meta" for p in parent.parameters(recurse=False)):
            raise RuntimeError(
                f"sync_sharded_amax: {name} receives another rank's pre_quant_scale but its module holds "
                "real weights; non-owned layers must be on the meta device (the owner folded 1/s into its own)"
            )
    off = 0
    for k, sz in zip(keys, sizes):
        (name, attr), (shape, dt) = k, layout[k]
        val = flat[off : off + sz].view(shape).to(getattr(torch, dt))
        q = mods.get(name)
        off += sz
        if q is None or k in mine:
            continue
        if attr == "_amax":
            if hasattr(q, "_amax"):
                delattr(q, "_amax")  # a meta placeholder from weight-only calibration
            q.amax = val
        else:
            if attr in q._buffers:
                del q._buffers[attr]
            q._enable_pre_quant_scale = True
            q.pre_quant_scale = val
    promote_static_block_weight_quantizers(model)
    return total
