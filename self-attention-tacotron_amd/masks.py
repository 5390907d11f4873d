"""Training-mode randomness of the hot path, as explicit mask tensors.

The reference draws dropout / zoneout noise inside TF ops (``tf.layers.dropout`` in PreNet and in
ScaledDotProductAttentionMechanism ``modules/self_attention.py:60``; ``tf.nn.dropout`` inside the
external ZoneoutLSTMCell).  Here every such draw is a mask tensor produced on the GPU by one
counter-based RNG launch (``sat_rng_fill``) per training step, so the oracle can be fed the SAME
masks for parity and the backward pass re-uses them without re-drawing.

Mask values:
* dropout  ("dropout"): 0 or 1/keep  (inverted dropout, applied by multiplication);
* zoneout  ("zoneout"): 1 = take the new state, 0 = keep the previous one (keep prob 1-z).

Layouts are batch-major for per-frame dropout and step-major ([T, B, U]) for recurrent state, the
order the recurrent kernels consume them.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

from .params import resolve_dims


@dataclass(frozen=True)
class MaskSpec:
    name: str
    shape: Tuple[int, ...]
    kind: str          # dropout | zoneout
    rate: float        # drop rate (dropout) or zoneout factor


def mask_specs(hp, B: int, N: int, Tp: int) -> List[MaskSpec]:
    d = resolve_dims(hp)
    out: List[MaskSpec] = []
    for i, u in enumerate(d.enc_prenet):
        out.append(MaskSpec(f"enc/prenet{i}", (B, N, u), "dropout", hp.encoder_prenet_drop_rate))
    zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
    for dr in ("fw", "bw"):
        out.append(MaskSpec(f"enc/lstm_{dr}/zc", (N, B, d.cbhg_half), "zoneout", zc))
        out.append(MaskSpec(f"enc/lstm_{dr}/zh", (N, B, d.cbhg_half), "zoneout", zh))
    for h in range(d.enc_hops):
        out.append(MaskSpec(f"enc/sa{h}/probs", (B, d.enc_heads, N, N), "dropout",
                            hp.self_attention_drop_rate))
    for i, u in enumerate(d.dec_prenet):   # step-major like every decoder-loop tensor
        out.append(MaskSpec(f"dec/prenet{i}", (Tp, B, u), "dropout", hp.decoder_prenet_drop_rate))
    for name, units in (("lstm0", d.att_rnn), ("lstm1", d.dec), ("lstm2", d.dec)):
        out.append(MaskSpec(f"dec/{name}/zc", (Tp, B, units), "zoneout", zc))
        out.append(MaskSpec(f"dec/{name}/zh", (Tp, B, units), "zoneout", zh))
    for h in range(d.dec_hops):
        out.append(MaskSpec(f"dec/sa{h}/probs", (B, d.dec_heads, Tp, Tp), "dropout",
                            hp.decoder_self_attention_drop_rate))
    return out
