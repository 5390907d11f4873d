"""Speed-of-light split (full / no DMA / no epilogue / neither) of the conv (implicit im2col)
products vs a dense product of the same size, and of the fused conv bank.
python tools/probes/conv_sol.py"""
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


def sol(name, f, fl):
    row = []
    for mode in (0, 1, 2, 3):
        lib.sat_gemm_probe_mode(mode)
        row.append(timeit(f))
    lib.sat_gemm_probe_mode(0)
    print(f"{name:40s} full {row[0]:7.1f} noDMA {row[1]:7.1f} noEpi {row[2]:7.1f} neither "
          f"{row[3]:7.1f} us  {fl / row[0] / 1e6:6.1f} TF/s (bound {fl / 157.3e6:.1f} us)", flush=True)


x = torch.randn(32, 200, 128, device="cuda")
for taps in (16, 8, 1):
    W = torch.randn(taps, 128, 128, device="cuda")
    out = torch.empty(32, 200, 128, device="cuda")
    for plan in ((64, 64, 1), (128, 64, 1), (64, 64, 4)):
        lib.sat_gemm_force_plan(*plan)
        sol(f"conv1d taps={taps} plan {plan}", lambda: K.conv1d(x, W, out=out),
            2.0 * 6400 * 128 * 128 * taps)
    lib.sat_gemm_force_plan(0, 0, 0)
    a = torch.randn(6400, 128 * taps, device="cuda")
    sol(f"dense 6400x128x{128 * taps}", lambda: K.gemm(a, W.view(-1, 128), out), 2.0 * 6400 * 128 * 128 * taps)
Wb = torch.randn(128 * 128 * 136, device="cuda") * 0.01
y = torch.empty(32, 200, 2048, device="cuda")
fl = 2.0 * 6400 * 128 * 128 * 136
for plan in ((64, 64, 1), (64, 128, 1), (128, 64, 1), (128, 128, 1)):
    lib.sat_gemm_force_plan(*plan)
    sol(f"conv bank fwd plan {plan}", lambda: K.conv_bank(x, Wb, None, y, 16, 128), fl)
lib.sat_gemm_force_plan(0, 0, 0)
dx = torch.empty_like(x)
dW = torch.empty_like(Wb)
sol("conv bank bwd dx", lambda: K.conv_bank_bwd(x, Wb, y, 16, 128, dx=dx), fl)
sol("conv bank bwd dW", lambda: K.conv_bank_bwd(x, Wb, y, 16, 128, dW=dW), fl)
