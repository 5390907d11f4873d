"""Drive ONE sat_gemm shape repeatedly (GPU; for rocprofv3 --pmc passes):
    python tools/probes/gemm_one.py M N K [a_trans] [reps]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import _lib  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

M, N, Kd = (int(x) for x in sys.argv[1:4])
at = int(sys.argv[4]) if len(sys.argv) > 4 else 0
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
a = torch.randn(Kd, M, device="cuda").t() if at else torch.randn(M, Kd, device="cuda")
b = torch.randn(Kd, N, device="cuda")
c = torch.empty(M, N, device="cuda")
for _ in range(reps):
    K.gemm(a, b, c)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    K.gemm(a, b, c)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / reps * 1e3
print(f"M={M} N={N} K={Kd} at={at}: {us:.1f} us  {2 * M * N * Kd / us / 1e6:.1f} TF/s")
ref = a @ b
print("max rel err", float((c - ref).abs().max() / ref.abs().max()))
