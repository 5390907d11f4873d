"""Synthetic LJSpeech-shaped batches honouring the reference's batch/padding contract.

Contract restated from ``datasets/ljspeech/dataset.py``:
* mel normalised ``(mel - avg) / std`` (:131-132) -- synthetic bodies are drawn directly in the
  normalised domain, N(0, 1);
* ``r`` frames of silence (``silence_mel_level_db`` = -3.0) at head and tail (:134-135), length
  rounded up to a multiple of ``r`` (:137-154, padding also -3.0);
* ``done`` = [0 ... 0, 1] of length T_b / r (:157-158); ``spec_loss_mask`` = 1[T_b],
  ``binary_loss_mask`` = 1[T_b / r] (:161-162);
* batch padding (:264-281): mel -3.0, done 1, masks 0, ids 0.
Source ids are characters 1..70 (``preprocess/text.py:21-28``).

Shapes "max" (every utterance N=200 chars, T=1000 frames) and "ljs" (N_b ~ U{40..200},
T_b ~ min(T, round_up_r(5 N_b + 2r))) follow SURVEY.md section 8(d).
"""

from __future__ import annotations

from typing import Dict, Optional

import numpy as np


def _round_up(x: int, r: int) -> int:
    return (x + r - 1) // r * r


def synthetic_batch(hp, B: int, N: int = 200, T: int = 1000, seed: int = 0, shape: str = "max",
                    num_chars: int = 70) -> Dict[str, np.ndarray]:
    r = hp.outputs_per_step
    M = hp.num_mels
    sil = hp.silence_mel_level_db
    if T % r:
        raise ValueError("T must be a multiple of outputs_per_step")
    rng = np.random.default_rng(seed)
    if shape == "max":
        n_len = np.full(B, N, np.int64)
        t_len = np.full(B, T, np.int64)
    elif shape == "ljs":
        n_len = rng.integers(max(1, min(40, N)), N + 1, size=B).astype(np.int64)
        t_len = np.minimum(T, [_round_up(int(5 * n + 2 * r), r) for n in n_len]).astype(np.int64)
    else:
        raise ValueError(shape)
    n_max, t_max = int(n_len.max()), int(t_len.max())
    t_max = _round_up(t_max, r)
    src = np.zeros((B, n_max), np.int64)
    mel = np.full((B, t_max, M), sil, np.float32)
    mel_mask = np.zeros((B, t_max), np.float32)
    done = np.ones((B, t_max // r), np.float32)
    done_mask = np.zeros((B, t_max // r), np.float32)
    for b in range(B):
        src[b, :n_len[b]] = rng.integers(1, num_chars + 1, size=int(n_len[b]))
        tb = int(t_len[b])
        body = rng.standard_normal((tb, M)).astype(np.float32)
        body[:r] = sil
        body[tb - r:] = sil
        mel[b, :tb] = body
        mel_mask[b, :tb] = 1.0
        done[b, :tb // r - 1] = 0.0
        done[b, tb // r - 1] = 1.0
        done_mask[b, :tb // r] = 1.0
    out = {"source": src, "source_length": n_len, "mel": mel, "mel_mask": mel_mask,
           "done": done, "done_mask": done_mask, "target_length": t_len}
    if hp.use_speaker_embedding:
        lo = hp.speaker_embedding_offset
        out["speaker_id"] = rng.integers(lo, lo + hp.num_speakers, size=B).astype(np.int64)
    return out


def synthetic_masks(hp, B: int, N: int, Tp: int, seed: int = 0,
                    only: Optional[set] = None) -> Dict[str, np.ndarray]:
    """Host-side (numpy) masks, for CPU tests of the mask plumbing.  The GPU path draws its
    masks with ``sat_rng_fill``; parity tests copy those to the oracle instead."""
    from .masks import mask_specs
    rng = np.random.default_rng(seed)
    out = {}
    for s in mask_specs(hp, B, N, Tp):
        if only is not None and s.name not in only:
            continue
        keep = 1.0 - s.rate
        u = rng.random(s.shape)
        if s.kind == "dropout":
            out[s.name] = np.where(u < keep, 1.0 / keep, 0.0).astype(np.float32)
        else:
            out[s.name] = (u < keep).astype(np.float32)
    return out
