"""Training step driver: masks -> forward -> BPTT -> (RCCL all-reduce) -> clip + Adam.

Host equivalent of the reference's TRAIN branch of ``model_fn`` (models/models.py:175-205) as
run by ``tf.estimator.train_and_evaluate`` (train.py:31-87), plus the data-parallel reduction
of ``MirroredStrategy`` (train.py:67,73).  One process per GPU: gradients are reduced over the
ONE flat gradient arena with a single ``torch.distributed.all_reduce`` (backend ``nccl`` ==
RCCL on ROCm, over xGMI), then clipped by global norm and applied -- every rank applies the same
update, so replicas stay bit-identical.

Reduction order: the build averages raw gradients across ranks and then clips (standard
synchronous data parallel).  TF1 MirroredStrategy clipped each replica's gradients before its
cross-replica reduction (models/models.py:183-189; the exact TF1 aggregation is
version-dependent) -- a documented deviation.

The whole step (mask RNG, forward, backward, optimiser) is capturable as one hipGraph: every
per-step varying scalar (RNG seed, global step, lr, clip scale) lives in device memory.
"""

from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from . import dp
from . import kernels as K
from .masks import mask_specs


class Trainer:
    def __init__(self, model, B: int, N: int, Tp: int, seed: int = 1234,
                 process_group=None, force_exchange: bool = False,
                 bucketed: Optional[bool] = None):
        self.m = model
        hp = model.hp
        dev = model.device
        self.hp = hp
        self.exp_avg = torch.zeros_like(model.params)
        self.exp_avg_sq = torch.zeros_like(model.params)
        self.global_step = torch.zeros(1, dtype=torch.int64, device=dev)
        self.seed = torch.tensor([seed], dtype=torch.int64, device=dev)
        self.scalars = torch.zeros(4, dtype=torch.float32, device=dev)
        # guarded update: {skipped steps, first error code} on the device; a pinned host mirror
        # refreshed after every step is inspected at the start of the next (no sync)
        self.status = torch.zeros(2, dtype=torch.int32, device=dev)
        self._mirror = torch.zeros(2 + model.health.numel(), dtype=torch.int32,
                                   pin_memory=torch.cuda.is_available())
        self._mirror_evt = None
        self.adam_ws = torch.empty(int(_lib.load().sat_workspace_adam()), dtype=torch.uint8,
                                   device=dev)
        self.cfg = _lib.SatAdamConfig()
        self.cfg.lr0 = hp.initial_learning_rate
        self.cfg.beta1, self.cfg.beta2, self.cfg.eps = hp.adam_beta1, hp.adam_beta2, hp.adam_eps
        self.cfg.clip_norm = 1.0
        self.cfg.decay = 1 if hp.decay_learning_rate else 0
        self.cfg.step_factor = hp.learning_rate_step_factor
        # every mask is a view of ONE arena, re-viewed when the batch shape changes (grown only
        # when a larger shape arrives), so a stream of differently padded batches keeps device
        # memory flat
        self._mask_arena = torch.empty(0, device=dev)
        self.shape = None
        self.reshape(B, N, Tp)
        self.pg = process_group
        self.world = dp.world_size(process_group)
        # run dp.exchange even in a one-rank group (tests of the RCCL path on one GPU)
        self.force_exchange = force_exchange
        self.cfg.grad_scale = dp.grad_scale(process_group)
        self.last_loss = None
        # bucketed exchange (SAT_DP_BUCKETS=1 / bucketed=True): the decoder's gradient rows are
        # all-reduced on a comm stream as soon as the decoder backward has issued them, beside
        # the encoder backward (inside the captured forward/backward graph in split replay);
        # the rest of the arena (encoder rows, BN statistics, health words) at the step's end.
        # Off by default: measured on one rank only (tests/test_dp_gpu.py), not on 8 GPUs.
        import os
        self.bucketed = (os.environ.get("SAT_DP_BUCKETS", "0") == "1" if bucketed is None
                         else bool(bucketed))
        self._comm = (torch.cuda.Stream(device=dev) if torch.device(dev).type == "cuda"
                      and self.bucketed else None)
        self._bucket_done = None

    def reshape(self, B: int, N: int, Tp: int) -> None:
        """Point the mask views at a (B, N, T') batch shape."""
        if self.shape == (B, N, Tp):
            return
        self.specs = mask_specs(self.hp, B, N, Tp)
        # every mask starts on a 256-byte boundary (64 floats): the fused attention kernels take
        # 16-byte-aligned operands only, and a segment packed right behind an odd-sized one
        # (e.g. B * N odd) would otherwise start misaligned.  Each segment's draw depends only
        # on its own stream id and index, so the padding changes no mask value.
        def up(n: int) -> int:
            return (n + 63) // 64 * 64
        need = sum(up(int(np.prod(s.shape))) for s in self.specs)
        if need > self._mask_arena.numel():
            self._mask_arena = torch.empty(need, device=self.m.device)
        self.masks: Dict[str, torch.Tensor] = {}
        off = 0
        segs = []
        for i, s in enumerate(self.specs):
            n = int(np.prod(s.shape))
            self.masks[s.name] = self._mask_arena[off:off + n].view(s.shape)
            keep = 1.0 - s.rate
            on = 1.0 / keep if s.kind == "dropout" else 1.0
            segs.append((off, n, i + 1, keep, on))
            off += up(n)
        self._mask_segs = K.rng_segments(segs)
        self.shape = (B, N, Tp)

    def draw_masks(self):
        """All masks in ONE Philox launch over the mask arena (sat_rng_fill_segments); each
        mask keeps its fixed stream id, so it is bit-identical to its own sat_rng_fill launch;
        the seed advances on the device every step."""
        K.rng_fill_segments(self._mask_arena, self._mask_segs, self.seed)

    def _bucketing(self) -> bool:
        return self.bucketed and (self.world > 1 or
                                  (self.force_exchange and dp.is_distributed(self.pg)))

    def _decoder_bucket(self, streams):
        """model_backward's on_decoder_grads hook: the first bucket's collective, on the comm
        stream once every stream that carried decoder-gradient work has reached this point."""
        lo, hi = self.m.decoder_grad_span()
        if self._comm is not None:
            for st in streams:
                self._comm.wait_stream(st)
            with torch.cuda.stream(self._comm):
                dp.exchange_bucket(self.m.exchange, lo, hi, self.pg, force=self.force_exchange)
        else:
            dp.exchange_bucket(self.m.exchange, lo, hi, self.pg, force=self.force_exchange)
        self._bucket_done = (lo, hi)

    def forward_backward(self, batch):
        self.draw_masks()
        out, sv = self.m.forward(batch, self.masks, training=True)
        self._bucket_done = None
        self.m.backward(sv, on_decoder_grads=self._decoder_bucket if self._bucketing() else None)
        if self._bucket_done is not None and self._comm is not None:
            torch.cuda.current_stream().wait_stream(self._comm)   # joined (graph capture too)
        self.last_loss = out["loss"]
        self.last_saved = sv
        return out

    def reduce_grads(self):
        """The step's ONE collective (dp.exchange): a SUM all-reduce of the engine's exchange
        arena -- gradients (1/world folded into Adam), the BatchNorm moving statistics
        (averaged, so replicas never drift apart) and the health words (non-zero everywhere iff
        on some rank, so the guarded update is skipped on every rank or on none)."""
        dp.exchange(self.m.exchange, self.m.health, self.m.bn.buf, self.m.health_tail, self.pg,
                    force=self.force_exchange, done=self._bucket_done)

    def apply(self):
        """Guarded clip + Adam: skipped on the device when any health word of the step is set."""
        m = self.m
        _lib.check(_lib.load().sat_adam_step(
            m.params.data_ptr(), m.grads.data_ptr(), self.exp_avg.data_ptr(),
            self.exp_avg_sq.data_ptr(), m.params.numel(), self.global_step.data_ptr(),
            self.scalars.data_ptr(), self.adam_ws.data_ptr(), _lib.ctypes.byref(self.cfg),
            m.health.data_ptr(), m.health.numel(), self.status.data_ptr(),
            K._stream()), "sat_adam_step")
        _lib.call("sat_counter_add", self.seed.data_ptr(), 1, K._stream())

    # ---- health: the previous step's verdict, read from pinned memory without a sync
    def publish_health(self):
        """Queue the copy of {status, health words} to the pinned mirror (outside graphs)."""
        self._mirror[:2].copy_(self.status, non_blocking=True)
        self._mirror[2:].copy_(self.m.health, non_blocking=True)
        self._mirror_evt = torch.cuda.Event()
        self._mirror_evt.record()

    def check_health(self, wait: bool = False):
        """Raise SatLibraryError if a finished step was skipped by the guard (``wait`` blocks
        until the last published step is done)."""
        if self._mirror_evt is None:
            return
        if wait:
            self._mirror_evt.synchronize()
        elif not self._mirror_evt.query():
            return
        if int(self._mirror[0]) != 0:
            self.m.raise_on_health(self._mirror[2:].tolist())
            raise _lib.SatLibraryError(
                f"{int(self._mirror[0])} training step(s) skipped by the health guard "
                f"(first error code {int(self._mirror[1])})")

    def step(self, batch):
        self.check_health()
        B, N = batch["source"].shape
        self.reshape(B, N, batch["mel"].shape[1] // self.hp.outputs_per_step)
        out = self.forward_backward(batch)
        self.reduce_grads()
        self.apply()
        self.publish_health()
        return out


class GraphedStep:
    """Capture Trainer.step (or its forward/backward half when an eager collective sits in
    between) into hipGraphs and replay them: kills the ~5k host launches per step."""

    def __init__(self, trainer: Trainer, batch, warmup: int = 1, split: Optional[bool] = None):
        """``split`` (default: world > 1) captures forward/backward and clip + Adam as two
        graphs with ``trainer.reduce_grads`` (the eager RCCL all-reduce) replayed between
        them."""
        self.t = trainer
        self.batch = batch
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        self.warm_out = None                    # the last warm-up step's output (a real step)
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.warm_out = trainer.step(batch)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.split = trainer.world > 1 if split is None else bool(split)
        self.g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fb):
            self.out = trainer.forward_backward(batch)
            if not self.split:
                trainer.apply()
        if self.split:
            self.g_apply = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_apply):
                trainer.apply()
        torch.cuda.synchronize()
        # the graph holds raw pointers into the grow-only buffers the step used (the mask
        # arena, the persistent kernels' scratch, the column-reduce / split-K / loss scratch):
        # keep those exact buffers alive for the graph's lifetime, so a later, larger shape
        # that replaces one of them (eager or another graph) never leaves this graph pointing
        # at freed memory
        m = trainer.m
        self._keep = [trainer._mask_arena, *m._scratch.values(), *m.ws.bufs.values(),
                      *K._SCRATCH.values(), *K._GEMM_WS.values()]

    def replay(self):
        self.t.check_health()
        self.g_fb.replay()
        if self.split:
            self.t.reduce_grads()
            self.g_apply.replay()
        self.t.publish_health()
        return self.out


class StepGraphCache:
    """The drop-in training path's graph cache (``model_fn`` TRAIN over the reference's
    bucketed, per-batch padded batches: datasets/ljspeech/dataset.py:235-286, train.py:39-65):
    one captured step (``GraphedStep``) per padded batch shape, bounded LRU.

    A shape seen for the first time runs its step eagerly -- the warm-up of its capture, a
    real training step on that batch -- and is then captured; every later batch of that shape
    is copied into the graph's static input buffers and replayed (one launch instead of ~225
    from Python).  The least recently used graph is dropped beyond ``size`` entries (its
    private memory pool goes with it); ``size = 0`` is the eager path.  Replays are bit-identical
    to eager steps on the same batches (``tests/test_train_gpu.py``).

    ``t_quantum`` > 0 pads T' (decoder steps) up to a multiple of it before the lookup, so
    batches whose longest utterance differs by a few frames share a graph: the padding is the
    reference's own batch padding (mel -3.0 -- masked, done 1 -- masked, both loss masks 0;
    datasets/ljspeech/dataset.py:264-281), so the loss and every gradient are unchanged in exact
    arithmetic (the padded steps carry zero loss seeds and the decoder head is causal); only the
    dropout / zoneout draws of batch-major masks shift.  Default 0: exact shapes, bitwise ==
    eager."""

    def __init__(self, trainer: Trainer, size: int = 8, t_quantum: int = 0):
        from collections import OrderedDict
        self.t = trainer
        self.size = int(size)
        self.t_quantum = int(t_quantum)
        self.entries: "OrderedDict[tuple, tuple]" = OrderedDict()
        self.hits = self.misses = self.evictions = 0

    def _pad_t(self, batch):
        q = self.t_quantum
        r = self.t.hp.outputs_per_step
        Tp = batch["mel"].shape[1] // r
        Tq = -(-Tp // q) * q if q > 0 else Tp
        if Tq == Tp:
            return batch
        pad = (Tq - Tp)
        out = dict(batch)
        B = batch["mel"].shape[0]
        dev = batch["mel"].device
        out["mel"] = torch.cat([batch["mel"], torch.full((B, pad * r, batch["mel"].shape[2]), -3.0,
                                                         device=dev)], 1)
        out["mel_mask"] = torch.cat([batch["mel_mask"], torch.zeros(B, pad * r, device=dev)], 1)
        out["done"] = torch.cat([batch["done"], torch.ones(B, pad, device=dev)], 1)
        out["done_mask"] = torch.cat([batch["done_mask"], torch.zeros(B, pad, device=dev)], 1)
        return out

    @staticmethod
    def key(batch):
        return tuple(sorted((k, tuple(v.shape), v.dtype) for k, v in batch.items()))

    def step(self, batch):
        """One training step on ``batch`` (device tensors); returns {"loss": a tensor that this
        cache does not overwrite later}."""
        if self.size <= 0:
            return {"loss": self.t.step(batch)["loss"]}
        batch = self._pad_t(batch)
        k = self.key(batch)
        e = self.entries.get(k)
        if e is None:
            self.misses += 1
            static = {n: v.clone() for n, v in batch.items()}
            g = GraphedStep(self.t, static, warmup=1)     # this batch's step = the warm-up
            self.entries[k] = (static, g)
            while len(self.entries) > self.size:
                self.entries.popitem(last=False)
                self.evictions += 1
            return {"loss": g.warm_out["loss"]}
        self.hits += 1
        self.entries.move_to_end(k)
        static, g = e
        for n, v in batch.items():
            static[n].copy_(v, non_blocking=True)
        # GraphedStep.replay() leaves Trainer.shape alone: the next eager step re-views the
        # masks for its own shape (Trainer.reshape), the captured graph keeps its own views
        out = g.replay()
        return {"loss": out["loss"].clone()}

