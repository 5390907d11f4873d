"""Chunked multi-stream schedule for the decoder's three recurrences.

Teacher forcing makes the decoder a stack of three recurrences with a one-way dependency per
step: attention RNN (+ dual-source attention) -> decoder LSTM1 -> decoder LSTM2 (forward), and
the reverse in BPTT.  Each recurrence is a chain of small latency-bound launches that leaves
most of the 256 CUs idle, so the build runs them as a software pipeline over chunks of decoder
steps: lane 0 = the current (capturing) stream, lanes 1 and 2 = two side HIP streams.  Chunk k
of lane i+1 waits on an event recorded after chunk k of lane i; the whole thing is captured as
one multi-stream hipGraph (events become graph edges).  With ``chunk == 0`` every lane is the
current stream and the same code runs strictly in program order (the reference schedule used by
the parity tests).
"""

from __future__ import annotations

import contextlib
from typing import List, Optional, Tuple

import torch


class Pipeline:
    def __init__(self, device, chunk: int = 25):
        self.chunk = int(chunk)
        self.device = torch.device(device)
        self.side: Optional[Tuple[torch.cuda.Stream, torch.cuda.Stream]] = None
        if self.chunk > 0 and self.device.type == "cuda":
            self.side = (torch.cuda.Stream(self.device), torch.cuda.Stream(self.device))

    @property
    def enabled(self) -> bool:
        return self.side is not None

    def chunks(self, T: int) -> List[Tuple[int, int]]:
        if not self.enabled:
            return [(0, T)]
        return [(a, min(T, a + self.chunk)) for a in range(0, T, self.chunk)]

    def fork(self):
        """Side lanes start after everything already queued on the current stream."""
        if self.enabled:
            main = torch.cuda.current_stream(self.device)
            for s in self.side:
                s.wait_stream(main)

    def join(self):
        if self.enabled:
            main = torch.cuda.current_stream(self.device)
            for s in self.side:
                main.wait_stream(s)

    def lane(self, i: int):
        """Context manager running the enclosed launches on lane i (0 = current stream)."""
        if not self.enabled or i == 0:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.side[i - 1])

    def _stream(self, i: int):
        return torch.cuda.current_stream(self.device) if i == 0 else self.side[i - 1]

    def handoff(self, src: int, dst: int):
        """Work queued on lane dst from now on waits for what lane src has queued so far."""
        if self.enabled:
            ev = torch.cuda.Event()
            ev.record(self._stream(src))
            self._stream(dst).wait_event(ev)


SEQUENTIAL = Pipeline("cpu", chunk=0)
