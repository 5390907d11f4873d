"""The conv bank's two backward products (dX and dW, B=32 x 200 positions, 16 banks x 128) timed
alone per forced LDS plan, and both at once on two streams -- what a joint launch could gain.
python tools/probes/convbank_bwd_probe.py"""
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
Wb = torch.randn(128 * 128 * 136, device="cuda") * 0.01
y = torch.randn(32, 200, 2048, device="cuda")
dx = torch.empty_like(x)
dW = torch.empty_like(Wb)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


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


def fdx():
    K.conv_bank_bwd(x, Wb, y, 16, 128, dx=dx)


def fdw():
    K.conv_bank_bwd(x, Wb, y, 16, 128, dW=dW)


def both():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        fdx()
    with torch.cuda.stream(s2):
        fdw()
    cur.wait_stream(s1)
    cur.wait_stream(s2)


fl = 2.0 * 6400 * 128 * 128 * 136
print("both products on two streams, per forced plan (the plan applies to both):", flush=True)
for plan in ((0, 0, 0), (64, 64, 3), (64, 128, 2)):
    lib.sat_gemm_force_plan(*plan)
    try:
        a, b = t_of(fdx), t_of(fdw)
        c = t_of(both)
    except Exception as e:  # noqa: BLE001  (a forced plan the scratch cannot take)
        print(f"plan {plan}: {e}", flush=True)
        continue
    print(f"plan {plan}: dX {a:7.1f} us ({fl / a / 1e6:5.1f} TF/s)  dW {b:7.1f} us "
          f"({fl / b / 1e6:5.1f} TF/s)  serial {a + b:7.1f}  two streams {c:7.1f}", flush=True)
print("each product alone, per forced plan:", flush=True)
for plan in ((128, 128, 1), (128, 128, 2), (128, 128, 3), (128, 128, 4), (128, 128, 6),
             (128, 128, 8), (128, 64, 3), (128, 64, 4), (64, 128, 3), (64, 128, 4)):
    lib.sat_gemm_force_plan(*plan)
    row = []
    for nm, f in (("dX", fdx), ("dW", fdw)):
        try:
            t = t_of(f)
            row.append(f"{nm} {t:7.1f} us ({fl / t / 1e6:5.1f} TF/s)")
        except Exception:  # noqa: BLE001
            row.append(f"{nm} (plan refused)")
    print(f"plan {plan}: " + "  ".join(row), flush=True)
lib.sat_gemm_force_plan(0, 0, 0)
