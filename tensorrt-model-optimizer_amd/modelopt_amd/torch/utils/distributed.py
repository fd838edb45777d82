"""Process-group wrappers used by calibration (reference: modelopt/torch/utils/distributed.py:398-466).

``None`` = the default (world) group, ``-1`` = disabled.  The amax exchange runs over whatever
backend torch.distributed was initialised with: ``nccl`` (= RCCL over xGMI on MI355X) for GPU
tensors, ``gloo`` in the CPU tests.
"""

from __future__ import annotations

import torch
import torch.distributed as dist

__all__ = ["DistributedProcessGroup", "ParallelState", "is_initialized", "size", "rank"]


def is_available() -> bool:
    return dist.is_available()


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def size(group=None) -> int:
    return dist.get_world_size(group) if is_initialized() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if is_initialized() else 0


class DistributedProcessGroup:
    """A process group that may be disabled (``-1``) or the default world group (``None``)."""

    def __init__(self, group=None):
        self.group = group

    def is_initialized(self) -> bool:
        return is_initialized() and self.group != -1

    def rank(self) -> int:
        return dist.get_rank(self.group) if self.is_initialized() else 0

    def world_size(self) -> int:
        return dist.get_world_size(self.group) if self.is_initialized() else 1

    @staticmethod
    def get_dist_syncd_obj(obj, groups, op):
        """all_gather_object over the group(s), then reduce with ``op`` (reference :421-438)."""
        if not isinstance(groups, (list, tuple)):
            groups = [groups]
        objs = [obj]
        for g in groups:
            if g is None or not g.is_initialized():
                continue
            gathered = [None] * g.world_size()
            dist.all_gather_object(gathered, obj, group=g.group)
            objs = gathered
        return op(objs)

    def __repr__(self):
        return f"DistributedProcessGroup(group={self.group}, initialized={self.is_initialized()})"


def fixed_order_sum(t: torch.Tensor, group: DistributedProcessGroup) -> torch.Tensor:
    """Sum of ``t`` over the ranks of ``group`` in rank order, fp32, identical on every rank.

    An ``all_reduce(SUM/AVG)`` adds in an order the collective's algorithm picks (ring chunks on
    RCCL), so the float result can differ across runs and topologies, and gloo has no AVG.  The
    tensors reduced here are small (an AWQ ``act_scale`` is one [K] vector per linear, the losses
    11 floats): gather them all and add ``((t_0 + t_1) + t_2) + ...`` on every rank instead.
    Host-staged under gloo when ``t`` lives on a device."""
    if not group.is_initialized():
        return t
    dev = t.device
    x = t.detach().to(torch.float32)
    if dist.get_backend(group.group) == "gloo" and x.device.type != "cpu":
        x = x.cpu()
    parts = [torch.empty_like(x) for _ in range(group.world_size())]
    dist.all_gather(parts, x.contiguous(), group=group.group)
    acc = parts[0].clone()
    for p in parts[1:]:
        acc += p
    return acc.to(dev)


def fixed_order_sum_many(tensors: list[torch.Tensor], group: DistributedProcessGroup) -> list[torch.Tensor]:
    """``fixed_order_sum`` of many tensors with ONE collective: all are flattened into one fp32
    buffer (every rank must pass the same shapes in the same order), gathered once, summed in
    rank order and split back (fp32, each slice on its own tensor's device: a model spread over
    several GPUs keeps every linear's result where the linear lives).  AWQ-lite uses it for the
    act_scale / NaN flags of every linear after the caching pass and for every linear's losses
    after the search pass: two collectives per calibration instead of two or three per linear."""
    if not tensors:
        return []
    flat = torch.cat([t.detach().reshape(-1).to(device=tensors[0].device, dtype=torch.float32) for t in tensors])
    summed = fixed_order_sum(flat, group) if group.is_initialized() else flat
    out, off = [], 0
    for t in tensors:
        n = t.numel()
        out.append(summed[off : off + n].reshape(t.shape).to(t.device))
        off += n
    return out


class ParallelState:
    """Data / tensor / expert parallel groups of a module (reference :441-466)."""

    def __init__(self, data_parallel_group=None, tensor_parallel_group=-1, expert_model_parallel_group=-1):
        self.data_parallel_group = DistributedProcessGroup(data_parallel_group)
        self.tensor_parallel_group = DistributedProcessGroup(tensor_parallel_group)
        self.expert_model_parallel_group = DistributedProcessGroup(expert_model_parallel_group)

    def __repr__(self):
        return (
            f"data_parallel_group: {self.data_parallel_group}, tensor_parallel_group: "
            f"{self.tensor_parallel_group}, expert_model_parallel_group: {self.expert_model_parallel_group}"
        )


def barrier(group=None):
    if is_initialized():
        dist.barrier(group=group)


def all_reduce_max_(t: torch.Tensor, group=None) -> torch.Tensor:
    if is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t
