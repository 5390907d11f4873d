"""The model object: flat parameter / gradient arenas on the device + forward / backward.

This is the host-side equivalent of ``DualSourceSelfAttentionTacotronModel`` (models/models.py:20)
minus the tf.estimator plumbing: it owns the weights (one fp32 arena), their gradients (a second
arena of the same layout), the BatchNorm moving statistics and the reduction workspace.
"""

from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from . import kernels as K
from . import params as PR
from .backward import model_backward
from .model import BNState, model_forward
from .pipeline import Pipeline


class Tacotron:
    def __init__(self, hp, device, seed: int = 1234,
                 init_values: Optional[Dict[str, np.ndarray]] = None, attn_tile: int = 32,
                 pipeline_chunk: int = 40, persistent_decoder: bool = True):
        self.hp = hp
        self.d = PR.resolve_dims(hp)
        self.device = torch.device(device)
        self.layout = PR.Layout(PR.param_specs(hp))
        vals = init_values if init_values is not None else PR.init_params(hp, seed)
        self.params = torch.tensor(self.layout.pack(vals)).to(self.device)
        # the data-parallel exchange arena: [gradients | BN moving statistics | health tail],
        # so a replica's whole per-step exchange is ONE SUM all-reduce (dp.exchange)
        n_p, n_bn = self.params.numel(), BNState.numel(hp)
        self.exchange = torch.zeros(n_p + n_bn + self.N_HEALTH, device=self.device)
        self.grads = self.exchange[:n_p]
        self.P = self.layout.views(self.params)
        self.G = self.layout.views(self.grads)
        self.bn = BNState(hp, self.device, storage=self.exchange[n_p:n_p + n_bn])
        self.health_tail = self.exchange[n_p + n_bn:]
        self.ws = K.Workspace(self.device)
        self.attn_tile = attn_tile
        # wavefront schedule of the decoder recurrences (0 = layer by layer)
        self.pipe = Pipeline(self.device, pipeline_chunk)
        # attention chain of the decoder forward as one persistent launch (when eligible)
        self.persistent_decoder = persistent_decoder
        # one persistent-kernel scratch per batch size, sized for the largest N seen (a batch of
        # a smaller N runs in a prefix of it), so a stream of differently padded batches does
        # not grow device memory
        self._scratch = {}
        # health arena: int32 error words of one step -- [0:2] attention chain fwd, [2:4] / [4:6]
        # decoder LSTM stack fwd / bwd, [6:8] attention chain bwd, [8] embedding id range,
        # [9] speaker-embedding id range; read on the device by the guarded Adam step
        self.health = torch.zeros(self.N_HEALTH, dtype=torch.int32, device=self.device)

    N_HEALTH = 16
    HEALTH_WORDS = {0: "sat_decoder_attention_fwd hand-off timeout",
                    2: "sat_decoder_lstms_fwd hand-off timeout",
                    4: "sat_decoder_lstms_bwd hand-off timeout",
                    6: "sat_decoder_attention_bwd group-barrier timeout",
                    8: "embedding id out of range", 9: "speaker id out of range"}

    def scratch(self, B: int, N: int):
        sc = self._scratch.get(B)
        if sc is None or sc.N < N:
            sc = K.DecoderAttentionScratch(B, max(N, 0 if sc is None else sc.N), self.device,
                                           errs=self.health)
            self._scratch[B] = sc
        return sc

    # ------------------------------------------------------------------ steps
    def forward(self, batch: Dict[str, torch.Tensor], masks=None, training: bool = True,
                need_grad: bool = True):
        B, N = batch["source"].shape
        scratch = self.scratch(B, N) if self.persistent_decoder else None
        return model_forward(self.P, self.bn, self.hp, self.d, batch, masks, training, self.ws,
                             compute_grad_seeds=need_grad, attn_tile=self.attn_tile,
                             pipe=self.pipe, persistent=self.persistent_decoder,
                             scratch=scratch, health=self.health)

    def raise_on_health(self, words) -> None:
        """Raise SatLibraryError naming every set error word (host copy of the arena)."""
        bad = [f"{self.HEALTH_WORDS.get(i, f'word {i}')} (code {int(v)})"
               for i, v in enumerate(words) if int(v) != 0]
        if bad:
            from ._lib import SatLibraryError
            raise SatLibraryError("training step unhealthy: " + "; ".join(bad))

    def backward(self, saved, zero: bool = True, on_decoder_grads=None):
        if zero:
            K.fill_(self.grads)
        model_backward(self.P, self.G, self.hp, self.d, saved, self.ws, attn_tile=self.attn_tile,
                       pipe=self.pipe, on_decoder_grads=on_decoder_grads)

    def decoder_grad_span(self):
        """(lo, hi) of the gradient arena rows the decoder's backward writes: every parameter
        after the encoder's (params.param_specs order: embedding, encoder/..., then
        [speaker_embedding,] decoder/...), a contiguous 256-byte-aligned tail of the gradients.
        The first bucket of the bucketed data-parallel exchange (train.Trainer)."""
        first = next(p.name for p in self.layout.specs
                     if p.name != "embedding" and not p.name.startswith("encoder/"))
        return self.layout.offsets[first], self.params.numel()

    # ------------------------------------------------------------------ host views
    def params_dict(self) -> Dict[str, np.ndarray]:
        return self.layout.unpack(self.params.detach().cpu().numpy())

    def grads_dict(self) -> Dict[str, np.ndarray]:
        return self.layout.unpack(self.grads.detach().cpu().numpy())

    @property
    def num_params(self) -> int:
        return self.layout.num_params
