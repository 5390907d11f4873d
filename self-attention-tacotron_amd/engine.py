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
        self.grads = torch.zeros_like(self.params)
        self.P = self.layout.views(self.params)
        self.G = self.layout.views(self.grads)
        self.bn = BNState(hp, self.device)
        self.ws = K.Workspace(self.device)
        self.attn_tile = attn_tile
        # wavefront schedule of the decoder recurrences (0 = layer by layer)
        self.pipe = Pipeline(self.device, pipeline_chunk)
        # attention chain of the decoder forward as one persistent launch (when eligible)
        self.persistent_decoder = persistent_decoder
        self._scratch = {}

    # ------------------------------------------------------------------ steps
    def forward(self, batch: Dict[str, torch.Tensor], masks=None, training: bool = True,
                need_grad: bool = True):
        B, N = batch["source"].shape
        scratch = None
        if self.persistent_decoder:
            key = (B, N)
            if key not in self._scratch:
                self._scratch[key] = K.DecoderAttentionScratch(B, N, self.device)
            scratch = self._scratch[key]
        return model_forward(self.P, self.bn, self.hp, self.d, batch, masks, training, self.ws,
                             compute_grad_seeds=need_grad, attn_tile=self.attn_tile,
                             pipe=self.pipe, persistent=self.persistent_decoder,
                             scratch=scratch)

    def backward(self, saved, zero: bool = True):
        if zero:
            self.grads.zero_()
        model_backward(self.P, self.G, self.hp, self.d, saved, self.ws, attn_tile=self.attn_tile,
                       pipe=self.pipe)

    # ------------------------------------------------------------------ host views
    def params_dict(self) -> Dict[str, np.ndarray]:
        return self.layout.unpack(self.params.detach().cpu().numpy())

    def grads_dict(self) -> Dict[str, np.ndarray]:
        return self.layout.unpack(self.grads.detach().cpu().numpy())

    @property
    def num_params(self) -> int:
        return self.layout.num_params
