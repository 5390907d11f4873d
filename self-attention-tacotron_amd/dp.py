"""Data parallelism: one process per GPU, synchronous replicas over RCCL (``nccl`` backend).

The reference replicates the step with tf.distribute.MirroredStrategy (train.py:67,73); here it
is plain synchronous data parallelism, one process per GPU: every rank runs the full teacher-forced step on its own batch shard, the flat gradient arena
(one contiguous fp32 buffer, ~25 MB for LJSpeech) is SUM-all-reduced in ONE collective, and the
1/world averaging is folded into the fused clip+Adam kernel (``SatAdamConfig.grad_scale``), so
the clip norm is the norm of the averaged gradient, as on one device with the global batch.

Kept free of GPU calls so the same functions run under ``gloo`` in the CPU tests.
"""

from __future__ import annotations

import torch
import torch.distributed as tdist


def is_distributed(group=None) -> bool:
    return tdist.is_available() and tdist.is_initialized()


def world_size(group=None) -> int:
    return tdist.get_world_size(group) if is_distributed(group) else 1


def rank(group=None) -> int:
    return tdist.get_rank(group) if is_distributed(group) else 0


def broadcast_params(flat: torch.Tensor, group=None, src: int = 0) -> None:
    """Identical initial weights on every replica (one collective over the whole arena)."""
    if world_size(group) > 1:
        tdist.broadcast(flat, src, group=group)


def grad_scale(group=None) -> float:
    """Factor the optimiser applies to the SUM-reduced gradient arena."""
    return 1.0 / world_size(group)


def allreduce_grads(flat: torch.Tensor, group=None) -> None:
    """SUM all-reduce of the flat gradient arena in place (averaging happens in Adam)."""
    if world_size(group) > 1:
        tdist.all_reduce(flat, op=tdist.ReduceOp.SUM, group=group)


def combine_health(words: torch.Tensor, group=None) -> None:
    """MAX over replicas of the step's int32 health words, in place (before the optimiser).

    Each rank's persistent kernels raise their own error words (a hand-off timeout, an id out
    of range).  The gradient all-reduce has already mixed a bad rank's gradients into every
    replica, so the guarded Adam step must skip on EVERY rank or on none: with the words
    combined, all ranks skip together and all raise on their next ``check_health`` (instead of
    the healthy ranks applying the update and then blocking in the next collective)."""
    if world_size(group) > 1:
        tdist.all_reduce(words, op=tdist.ReduceOp.MAX, group=group)


def average_buffer(flat: torch.Tensor, group=None) -> None:
    """Mean over replicas in place (BatchNorm moving statistics: the replicas' updates are
    averaged each step so every rank holds the same EVAL / checkpoint state; TF1
    MirroredStrategy's exact aggregation of BN moving averages is unpinned)."""
    w = world_size(group)
    if w > 1:
        tdist.all_reduce(flat, op=tdist.ReduceOp.SUM, group=group)
        flat.mul_(1.0 / w)


def max_over_ranks(value: float, device, group=None) -> float:
    """The bench's step time: the slowest rank defines the job's throughput."""
    if world_size(group) == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX, group=group)
    return float(t.item())
