#!/usr/bin/env python3
"""Microbenchmark: cost per dependent kernel launch on this stack (eager vs hipGraph replay),
using the 1-thread sat_counter_add kernel of libsat_hip."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402
from sat_amd import _lib, kernels as K  # noqa: E402

n = 2000
c = torch.zeros(1, dtype=torch.int64, device="cuda")


def burst():
    for _ in range(n):
        _lib.call("sat_counter_add", c.data_ptr(), 1, K._stream())


burst()
torch.cuda.synchronize()
t = time.perf_counter(); burst(); torch.cuda.synchronize()
print(f"eager : {(time.perf_counter() - t) / n * 1e6:.2f} us/launch")
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    burst()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    burst()
g.replay(); torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
print(f"graph : {(time.perf_counter() - t) / (5 * n) * 1e6:.2f} us/launch")
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record(); g.replay(); ev1.record(); torch.cuda.synchronize()
print(f"graph (events): {ev0.elapsed_time(ev1) * 1e3 / n:.2f} us/launch, counter={int(c.item())}")
