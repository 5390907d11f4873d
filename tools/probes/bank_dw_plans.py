"""The conv bank's weight-gradient product (M = 136 x 128 (conv, tap, channel) rows, N = 128,
K = 32 x 200 positions) per forced LDS plan, alone and beside the input-gradient product (its
own plan) on a second stream -- the way the step runs them.
python tools/probes/bank_dw_plans.py"""
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
fl = 2.0 * 6400 * 128 * 128 * 136


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


DX_PLAN = [(0, 0, 0)]


def fdx():
    lib.sat_gemm_force_plan(*DX_PLAN[0])
    K.conv_bank_bwd(x, Wb, y, 16, 128, dx=dx)
    lib.sat_gemm_force_plan(0, 0, 0)


def make_fdw(plan):
    def f():
        lib.sat_gemm_force_plan(*plan)
        K.conv_bank_bwd(x, Wb, y, 16, 128, dW=dW)
        lib.sat_gemm_force_plan(0, 0, 0)
    return f


def both(fdw):
    def f():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s2):
            fdw()
        with torch.cuda.stream(s1):
            fdx()
        cur.wait_stream(s1)
        cur.wait_stream(s2)
    return f


if len(sys.argv) > 1 and sys.argv[1] == "joint":
    for pw in ((0, 0, 0), (128, 128, 2), (64, 128, 2), (128, 64, 2)):
        for px in ((0, 0, 0), (128, 128, 2), (128, 128, 3), (64, 128, 2), (64, 128, 4),
                   (128, 64, 4), (64, 64, 4)):
            DX_PLAN[0] = px
            try:
                a = t_of(fdx)
                c = t_of(both(make_fdw(pw)))
            except Exception as e:  # noqa: BLE001
                lib.sat_gemm_force_plan(0, 0, 0)
                print(f"dW {pw} dX {px}: {e}", flush=True)
                continue
            print(f"dW {pw} dX {px}: dX alone {a:7.1f} us  pair {c:7.1f} us", flush=True)
    sys.exit(0)
print(f"dX alone (its plan): {t_of(fdx):7.1f} us", flush=True)
for plan in ((0, 0, 0), (64, 64, 1), (64, 64, 2), (64, 64, 3), (64, 64, 4), (128, 64, 1),
             (128, 64, 2), (128, 64, 3), (128, 64, 4), (64, 128, 2), (64, 128, 3),
             (128, 128, 2), (128, 128, 3), (128, 128, 4), (128, 128, 6)):
    fdw = make_fdw(plan)
    try:
        torch.manual_seed(0)
        fdw()
        torch.cuda.synchronize()
        h = float(dW.double().abs().sum())
        a = t_of(fdw)
        c = t_of(both(fdw))
    except Exception as e:  # noqa: BLE001  (a forced plan the scratch cannot take)
        lib.sat_gemm_force_plan(0, 0, 0)
        print(f"plan {plan}: {e}", flush=True)
        continue
    print(f"plan {plan}: dW {a:7.1f} us ({fl / a / 1e6:5.1f} TF/s)  beside dX {c:7.1f} us  "
          f"|dW| {h:.6e}", flush=True)
