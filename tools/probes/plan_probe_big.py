"""Forced LDS-kernel tile plans for the step's large plain products -- the LSTM stack's input
projection (16000 x 1024 x 544), its input gradient (16000 x 544 x 1024), the head's projections
-- isolated, HIP events over 20 launches (GPU):  python tools/probes/plan_probe_big.py"""
import os, sys
sys.path.insert(0, os.getcwd())
import _sat_path
_sat_path.load()
import torch
from sat_amd import _lib, kernels as K
lib = _lib.load()
def t_of(f, reps=20):
    for _ in range(3): f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): f()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps
g = torch.Generator(device="cuda").manual_seed(1)
for (M, N, Kd, bt) in ((16000, 1024, 544, 1), (16000, 544, 1024, 0), (16000, 1024, 256, 1), (16000, 768, 256, 0)):
    a = torch.randn(M, Kd, device="cuda", generator=g)
    b = torch.randn(*((N, Kd) if bt else (Kd, N)), device="cuda", generator=g)
    B = b.t() if bt else b
    c = torch.empty(M, N, device="cuda")
    row = []
    for plan in ((0, 0, 0), (128, 64, 1), (64, 128, 1), (128, 128, 1), (64, 64, 1)):
        lib.sat_gemm_force_plan(*plan)
        try:
            row.append(f"{plan[:2]} {t_of(lambda: K.gemm(a, B, c)):6.1f}")
        finally:
            lib.sat_gemm_force_plan(0, 0, 0)
    print(f"{M}x{N}x{Kd} bt={bt}: " + " | ".join(row), flush=True)
