"""The decoder LSTM stack's input gradient d[h0' | c1 | c2] = dG1 W1[:544]^T (16000 x 544 x 1024,
backward.py dh0_chunk) as ONE product (C2 output split at 256) against two: the 512 columns that
fill 128 x 256 tiles (250 tiles, one round on 256 CUs) and the 32-column remainder.
python tools/probes/dh0_split_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import _lib  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

lib = _lib.load()
n, A, R0, G4 = 16000, 256, 288 + 32, 1024
dg = torch.randn(n, G4, device="cuda")
W1 = torch.randn(544 + 1024, G4, device="cuda") * 0.03
dH0 = torch.empty(n, A, device="cuda")
RD = torch.empty(n, R0, device="cuda")
side = torch.cuda.Stream()


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


def one():
    K.gemm(dg, W1[:544].t(), dH0, C2=RD[:, :288])


def forced(plan, f):
    def g():
        lib.sat_gemm_force_plan(*plan)
        try:
            f()
        finally:
            lib.sat_gemm_force_plan(0, 0, 0)
    return g


def main_part():
    K.gemm(dg, W1[:512].t(), dH0, C2=RD[:, :256])


def rest():
    K.gemm(dg, W1[512:544].t(), RD[:, 256:288])


def split_serial(plan):
    def g():
        forced(plan, main_part)()
        rest()
    return g


def split_side(plan):
    def g():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            rest()
        forced(plan, main_part)()
        cur.wait_stream(side)
    return g


one()
ref0, ref1 = dH0.clone(), RD[:, :288].clone()
print(f"one product call (the library plan; with the column split on, two launches): {t_of(one):7.1f} us", flush=True)
print(f"  remainder 16000 x 32 x 1024 alone: {t_of(rest):7.1f} us", flush=True)
for plan in ((128, 256, 1), (128, 128, 1), (64, 128, 1), (256, 128, 1)):
    try:
        a = t_of(forced(plan, main_part))
        b = t_of(split_serial(plan))
        c = t_of(split_side(plan))
    except Exception as e:  # noqa: BLE001
        print(f"plan {plan}: {e}", flush=True)
        continue
    e0 = float((dH0 - ref0).abs().max() / ref0.abs().max())
    e1 = float((RD[:, :288] - ref1).abs().max() / ref1.abs().max())
    print(f"plan {plan}: 512 columns {a:7.1f} us, + remainder serial {b:7.1f} us, remainder on a "
          f"side stream {c:7.1f} us  (rel diff vs one product {e0:.1e} / {e1:.1e})", flush=True)
for plan in ((64, 64, 1), (64, 64, 2), (64, 64, 4), (64, 64, 8), (128, 64, 4), (128, 64, 8)):
    try:
        print(f"remainder plan {plan}: {t_of(forced(plan, rest)):7.1f} us", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"remainder plan {plan}: {e}", flush=True)
