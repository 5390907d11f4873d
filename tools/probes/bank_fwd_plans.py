"""The fused conv-bank forward (C2 shape: 32 x 200 positions, 128 channels, 16 banks x 128) per
forced LDS tile shape, with the longest-first dispatch (GPU):
python tools/probes/bank_fwd_plans.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import _lib  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

lib = _lib.load()
x = torch.randn(32, 200, 128, device="cuda")
Wb = torch.randn(128 * 128 * 136, device="cuda") * 0.05
b = torch.randn(16 * 128, device="cuda")
y = torch.empty(32, 200, 2048, device="cuda")
fl = 2.0 * 6400 * 128 * 128 * 136


def t_of(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


ref = None
for plan in ((0, 0, 0), (64, 128, 1), (128, 128, 1), (128, 64, 1), (64, 64, 1)):
    lib.sat_gemm_force_plan(*plan)
    try:
        K.conv_bank(x, Wb, b, y, 16, 128)
        torch.cuda.synchronize()
        d = 0.0 if ref is None else float((y - ref).abs().max())
        if ref is None:
            ref = y.clone()
        t = t_of(lambda: K.conv_bank(x, Wb, b, y, 16, 128))
        print(f"plan {plan}: {t:7.1f} us  {fl / t / 1e6:6.1f} TF/s  max|diff| vs default {d:.3g}",
              flush=True)
    finally:
        lib.sat_gemm_force_plan(0, 0, 0)
