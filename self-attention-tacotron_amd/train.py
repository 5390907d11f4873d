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

import torch

from . import _lib
from . import dp
from . import kernels as K
from .masks import mask_specs


class Trainer:
    def __init__(self, model, B: int, N: int, Tp: int, seed: int = 1234,
                 process_group=None):
        self.m = model
        hp = model.hp
        dev = model.device
        self.hp = hp
        self.exp_avg = torch.zeros_like(model.params)
        self.exp_avg_sq = torch.zeros_like(model.params)
        self.global_step = torch.zeros(1, dtype=torch.int64, device=dev)
        self.seed = torch.tensor([seed], dtype=torch.int64, device=dev)
        self.scalars = torch.zeros(4, dtype=torch.float32, device=dev)
        self.adam_ws = torch.empty(int(_lib.load().sat_workspace_adam()), dtype=torch.uint8,
                                   device=dev)
        self.cfg = _lib.SatAdamConfig()
        self.cfg.lr0 = hp.initial_learning_rate
        self.cfg.beta1, self.cfg.beta2, self.cfg.eps = hp.adam_beta1, hp.adam_beta2, hp.adam_eps
        self.cfg.clip_norm = 1.0
        self.cfg.decay = 1 if hp.decay_learning_rate else 0
        self.cfg.step_factor = hp.learning_rate_step_factor
        self.specs = mask_specs(hp, B, N, Tp)
        self.masks: Dict[str, torch.Tensor] = {
            s.name: torch.empty(s.shape, device=dev) for s in self.specs}
        self.pg = process_group
        self.world = dp.world_size(process_group)
        self.cfg.grad_scale = dp.grad_scale(process_group)
        self.last_loss = None

    def draw_masks(self):
        """One Philox launch per mask tensor; stream ids are fixed per mask, the seed advances
        on the device every step."""
        for i, s in enumerate(self.specs):
            keep = 1.0 - s.rate
            on = 1.0 / keep if s.kind == "dropout" else 1.0
            K.rng_fill(self.masks[s.name], self.seed, i + 1, keep, on)

    def forward_backward(self, batch):
        self.draw_masks()
        out, sv = self.m.forward(batch, self.masks, training=True)
        self.m.backward(sv)
        self.last_loss = out["loss"]
        self.last_saved = sv
        return out

    def reduce_grads(self):
        dp.allreduce_grads(self.m.grads, self.pg)

    def apply(self):
        m = self.m
        _lib.check(_lib.load().sat_adam_step(
            m.params.data_ptr(), m.grads.data_ptr(), self.exp_avg.data_ptr(),
            self.exp_avg_sq.data_ptr(), m.params.numel(), self.global_step.data_ptr(),
            self.scalars.data_ptr(), self.adam_ws.data_ptr(), _lib.ctypes.byref(self.cfg),
            K._stream()), "sat_adam_step")
        _lib.call("sat_counter_add", self.seed.data_ptr(), 1, K._stream())

    def step(self, batch):
        out = self.forward_backward(batch)
        self.reduce_grads()
        self.apply()
        return out


class GraphedStep:
    """Capture Trainer.step (or its forward/backward half when an eager collective sits in
    between) into hipGraphs and replay them: kills the ~5k host launches per step."""

    def __init__(self, trainer: Trainer, batch, warmup: int = 1):
        self.t = trainer
        self.batch = batch
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                trainer.step(batch)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.split = trainer.world > 1
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

    def replay(self):
        self.g_fb.replay()
        if self.split:
            self.t.reduce_grads()
            self.g_apply.replay()
        return self.out
