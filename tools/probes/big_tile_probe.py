"""The 256 x 128 / 128 x 256 LDS-GEMM tiles (8 waves of 64 x 64, 2-stage ring) against the
current plans on the conv bank's input gradient (alone and beside its weight gradient on a
second stream, as in the training step) and on a few 16000-row products.
python tools/probes/big_tile_probe.py"""
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


def fdx(plan):
    lib.sat_gemm_force_plan(*plan)
    try:
        K.conv_bank_bwd(x, Wb, y, 16, 128, dx=dx)
    finally:
        lib.sat_gemm_force_plan(0, 0, 0)


def fdw():
    K.conv_bank_bwd(x, Wb, y, 16, 128, dW=dW)


def both(plan):
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        fdx(plan)
    with torch.cuda.stream(s2):
        fdw()
    cur.wait_stream(s1)
    cur.wait_stream(s2)


fl = 2.0 * 6400 * 128 * 128 * 136
ref = None
print("conv bank dX (GRP 2) per plan; dW at its own plan beside it", flush=True)
for plan in ((0, 0, 0), (256, 128, 1), (256, 128, 2), (256, 128, 3), (256, 128, 4), (256, 128, 6),
             (256, 128, 8), (128, 128, 4)):
    a = t_of(lambda: fdx(plan))
    out = dx.clone()
    if ref is None:
        ref = out
    err = float((out - ref).abs().max() / ref.abs().max())
    c = t_of(lambda: both(plan))
    print(f"plan {plan}: dX {a:7.1f} us ({fl / a / 1e6:5.1f} TF/s) rel {err:.1e}  with dW on a "
          f"second stream {c:7.1f} us", flush=True)
print(f"dW alone {t_of(fdw):7.1f} us", flush=True)

print("dense products per plan (us)", flush=True)
shapes = [(16000, 1024, 544, False, False), (16000, 544, 1024, False, True),
          (16000, 1024, 256, False, False), (16000, 1024, 128, False, False),
          (544, 1024, 16000, True, False), (256, 1024, 16000, True, False)]
plans = ((0, 0, 0), (256, 128, 1), (128, 256, 1), (128, 128, 1), (256, 128, 2), (128, 256, 2),
         (256, 128, 4), (128, 256, 4), (128, 256, 8), (128, 256, 16), (64, 64, 12))
for M, N, Kd, ta, tb in shapes:
    A = torch.randn(Kd, M, device="cuda") if ta else torch.randn(M, Kd, device="cuda")
    B = torch.randn(N, Kd, device="cuda") if tb else torch.randn(Kd, N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    Aop, Bop = (A.t() if ta else A), (B.t() if tb else B)
    exp = (Aop.double() @ Bop.double()) if M * N * Kd <= 16000 * 1024 * 1024 else None
    row = []
    for plan in plans:
        if plan[2] > 1 and Kd < 512:
            continue
        lib.sat_gemm_force_plan(*plan)
        try:
            t = t_of(lambda: K.gemm(Aop, Bop, C))
        except Exception:  # noqa: BLE001
            row.append(f"{plan[0]}x{plan[1]}/s{plan[2]}:refused")
            continue
        finally:
            lib.sat_gemm_force_plan(0, 0, 0)
        e = float(((C.double() - exp).abs().max() / exp.abs().max())) if exp is not None else 0.0
        row.append(f"{plan[0]}x{plan[1]}/s{plan[2]}:{t:.1f}" + ("" if e < 1e-5 else f"(ERR {e:.1e})"))
    print(f"{M}x{N}x{Kd} ta={int(ta)} tb={int(tb)}: " + " ".join(row), flush=True)
