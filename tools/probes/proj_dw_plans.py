"""The CBHG projection layers' weight-gradient products (proj1: im2col(mp [32, 200, 2048], 3
taps) ^T dY [6400, 128] -> [3, 2048, 128], 10 GF; proj2: [3, 128, 128], 0.6 GF) per forced LDS
plan, alone -- they end the step's backward tail on the side stream.
python tools/probes/proj_dw_plans.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import _lib  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

lib = _lib.load()


def t_of(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps


for name, cin in (("proj1", 2048), ("proj2", 128)):
    x = torch.randn(32, 200, cin, device="cuda")
    dy = torch.randn(32, 200, 128, device="cuda")
    dW = torch.zeros(3, cin, 128, device="cuda")
    fl = 2.0 * 6400 * 3 * cin * 128
    ref = None
    for plan in ((0, 0, 0), (64, 64, 1), (64, 64, 2), (64, 64, 4), (64, 64, 8), (128, 64, 1),
                 (128, 64, 2), (128, 64, 4), (128, 64, 8), (64, 128, 2), (64, 128, 4),
                 (128, 128, 2), (128, 128, 4), (128, 128, 8), (128, 128, 16)):
        def f(plan=plan):
            lib.sat_gemm_force_plan(*plan)
            K.conv1d_dw(x, dy, dW)
            lib.sat_gemm_force_plan(0, 0, 0)
        try:
            f()
            torch.cuda.synchronize()
            if ref is None:
                ref = dW.clone()
            err = float((dW - ref).abs().max())
            a = t_of(f)
        except Exception as e:  # noqa: BLE001
            lib.sat_gemm_force_plan(0, 0, 0)
            print(f"{name} plan {plan}: {e}", flush=True)
            continue
        print(f"{name} plan {plan}: {a:7.1f} us ({fl / a / 1e6:5.1f} TF/s)  max|d| {err:.2e}",
              flush=True)
