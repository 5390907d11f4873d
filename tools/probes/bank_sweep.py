"""Forced plans of the fused conv-bank launches (C2 encoder shape): python bank_sweep.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import _lib  # noqa: E402
from sat_amd import kernels as K  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

lib = _lib.load()
x = torch.randn(32, 200, 128, device="cuda")
Wb = torch.randn(128 * 128 * 136, device="cuda") * 0.01
y = torch.randn(32, 200, 2048, device="cuda")
dx = torch.empty_like(x)
dW = torch.empty_like(Wb)
for name, f in (("dx", lambda: K.conv_bank_bwd(x, Wb, y, 16, 128, dx=dx)),
                ("dW", lambda: K.conv_bank_bwd(x, Wb, y, 16, 128, dW=dW))):
    lib.sat_gemm_force_plan(0, 0, 0)
    auto = timeit(f)
    res = []
    for bm, bn in ((128, 128), (128, 64), (64, 128), (64, 64)):
        for sp in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32):
            lib.sat_gemm_force_plan(bm, bn, sp)
            try:
                res.append((timeit(f), bm, bn, sp))
            except Exception:
                pass
    lib.sat_gemm_force_plan(0, 0, 0)
    res.sort()
    print(name, f"auto {auto:.1f}", " ".join(f"{bm}x{bn}/s{s}:{us:.1f}" for us, bm, bn, s in res[:8]),
          flush=True)
