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


def _active(group, force: bool) -> bool:
    return world_size(group) > 1 or (force and is_distributed(group))


def exchange_bucket(arena: torch.Tensor, lo: int, hi: int, group=None,
                    force: bool = False) -> None:
    """The bucketed exchange's first collective: SUM all-reduce of ``arena[lo:hi]`` -- the
    decoder's gradient rows, final once the decoder backward is done, reduced (on a stream of
    the caller's) while the encoder backward runs.  Plain gradients: no pack / unpack; the
    rest of the arena follows in ``exchange(..., done=(lo, hi))``."""
    if not _active(group, force):
        return
    tdist.all_reduce(arena[lo:hi], op=tdist.ReduceOp.SUM, group=group)


def exchange(arena: torch.Tensor, health: torch.Tensor, bn: torch.Tensor, tail: torch.Tensor,
             group=None, force: bool = False, done=None) -> None:
    """A replica's whole per-step exchange as ONE SUM all-reduce over the contiguous arena
    ``[gradients | bn | tail]`` (``bn`` and ``tail`` are views of it):

    * gradients: summed (the 1/world averaging is folded into Adam's ``grad_scale``);
    * BatchNorm moving statistics: pre-scaled by 1/world, so the sum is the replicas' mean;
    * health words: sent as |code| floats in ``tail`` and read back as ints, so a word is
      non-zero on every rank iff it was on some rank (the guarded Adam step then skips on every
      rank or on none) and the code is exact when one rank failed.

    On device tensors the pack / unpack are the library's ``sat_exchange_pack/unpack``
    launches; the host arithmetic below is the same restatement for the ``gloo`` CPU tests.

    ``force`` runs the whole exchange (pack, collective, unpack) even in a one-rank group, where
    it is the identity: the GPU tests drive the RCCL path that way on a one-GPU box.

    ``done = (lo, hi)``: that gradient range was reduced already (``exchange_bucket``); the
    rest -- ``arena[:lo]`` and ``arena[hi:]`` (BN statistics and health tail included) -- is
    reduced here as two collectives.  Every element is the same rank-ordered SUM either way
    (bitwise equal to the single collective at world 2; at larger worlds the ring's per-chunk
    summation order may differ in the last bit)."""
    w = world_size(group)
    if not _active(group, force):
        return

    def reduce_all():
        if done is None:
            tdist.all_reduce(arena, op=tdist.ReduceOp.SUM, group=group)
            return
        lo, hi = done
        if lo > 0:
            tdist.all_reduce(arena[:lo], op=tdist.ReduceOp.SUM, group=group)
        tdist.all_reduce(arena[hi:], op=tdist.ReduceOp.SUM, group=group)
    if arena.is_cuda:
        from . import _lib
        from . import kernels as K
        lib = _lib.load()
        _lib.check(lib.sat_exchange_pack(health.data_ptr(), health.numel(), bn.data_ptr(),
                                         bn.numel(), tail.data_ptr(), 1.0 / w, K._stream()),
                   "sat_exchange_pack")
        reduce_all()
        _lib.check(lib.sat_exchange_unpack(tail.data_ptr(), health.numel(), health.data_ptr(),
                                           K._stream()), "sat_exchange_unpack")
        return
    tail[:health.numel()].copy_(health.abs().float())
    bn.mul_(1.0 / w)
    reduce_all()
    health.copy_(tail[:health.numel()].to(torch.int32))


def max_over_ranks(value: float, device, group=None) -> float:
    """The bench's step time: the slowest rank defines the job's throughput."""
    if world_size(group) == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX, group=group)
    return float(t.item())
