"""Wavefront schedule of the decoder's three recurrences (single HIP stream).

Teacher forcing makes the decoder a stack of three recurrences with a one-way dependency per
step: attention RNN (+ dual-source attention) -> decoder LSTM1 -> decoder LSTM2 (forward), and
the reverse in BPTT.  Each recurrence step is a latency-bound launch that leaves most CUs idle,
and on MI355X / ROCm 7.2 independent streams (or graph branches) do not overlap such launches
(measured: tools/concurrency_probe.py), so the overlap is built into the launches themselves:
iteration i issues ONE multi-problem LSTM launch holding the attention RNN at step i, LSTM1 at
step i - C and LSTM2 at step i - 2C (disjoint workgroup ranges, ``sat_lstm_steps_fwd``); the
LSTMs' input projections are hoisted per chunk of C steps into GEMMs issued as soon as the
producing layer has finished the chunk.  The backward runs the mirror image (LSTM2 at
T'-1-j, LSTM1 C steps behind, the attention chain 2C behind).

``chunk == 0`` selects the plain layer-by-layer order (the reference schedule of the parity
tests): same arithmetic per step, different launch grouping.
"""

from __future__ import annotations

from typing import Dict, List, Tuple


class Pipeline:
    def __init__(self, device=None, chunk: int = 25):
        self.chunk = int(chunk)

    @property
    def enabled(self) -> bool:
        return self.chunk > 0

    def chunks(self, T: int) -> List[Tuple[int, int]]:
        if not self.enabled:
            return [(0, T)]
        return [(a, min(T, a + self.chunk)) for a in range(0, T, self.chunk)]

    def finishing(self, T: int, lag: int) -> Dict[int, Tuple[int, int]]:
        """iteration -> chunk whose last step (forward order) runs at that iteration on the
        layer that lags the chain by ``lag`` steps."""
        return {b - 1 + lag: (a, b) for a, b in self.chunks(T)}

    def finishing_rev(self, T: int, lag: int) -> Dict[int, Tuple[int, int]]:
        """reverse-order twin: iteration j processes step T-1-j+lag... of a layer ``lag`` steps
        behind the first; the chunk [a, b) finishes when its first step a is processed."""
        return {T - 1 - a + lag: (a, b) for a, b in self.chunks(T)}


SEQUENTIAL = Pipeline(chunk=0)
