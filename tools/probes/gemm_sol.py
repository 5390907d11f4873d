"""Speed-of-light split of the LDS GEMM (EXPERIMENT): full / no DMA / no epilogue / neither,
per forced plan.  python tools/probes/gemm_sol.py"""
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
for M, N, Kd in [(16000, 1024, 256), (16000, 256, 1024), (16000, 1024, 1024)]:
    a = torch.randn(M, Kd, device="cuda")
    b = torch.randn(Kd, N, device="cuda")
    c = torch.empty(M, N, device="cuda")
    for plan in [(128, 128, 1), (128, 64, 1), (64, 64, 1)]:
        lib.sat_gemm_force_plan(*plan)
        row = []
        for mode in (0, 1, 2, 3):
            lib.sat_gemm_probe_mode(mode)
            row.append(timeit(lambda: K.gemm(a, b, c)))
        lib.sat_gemm_probe_mode(0)
        fl = 2.0 * M * N * Kd
        print(f"{M}x{N}x{Kd} plan {plan}: full {row[0]:.1f} noDMA {row[1]:.1f} noEpi {row[2]:.1f} "
              f"neither {row[3]:.1f} us   (MFMA-only bound {fl / 157.3e6:.1f} us)", flush=True)
lib.sat_gemm_force_plan(0, 0, 0)
