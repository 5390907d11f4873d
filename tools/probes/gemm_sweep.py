"""Sweep the LDS GEMM kernel's tile / split-K plans per shape (GPU):
    python tools/probes/gemm_sweep.py [--shapes census]
Prints, per shape, the planner's choice and every forced (BM, BN, S) plan's time (HIP events,
10 launches after 3 warm-ups) so the cost model in gemm.hip:launch_lds can be checked."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import _lib  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

# (M, N, K, a_trans, b_trans) dense shapes of the step (tools/gemm_census.py), conv shapes as
# ("conv", S*L, Ci, taps, Co)
SHAPES = [
    (16000, 256, 256, 0, 0), (16000, 256, 256, 0, 1), (16000, 1024, 288, 0, 1),
    (16000, 288, 1024, 0, 0), (16000, 1024, 256, 0, 1), (16000, 256, 1024, 0, 0),
    (16000, 1024, 128, 0, 1), (16000, 128, 1024, 0, 0), (256, 1024, 16000, 1, 0),
    (544, 1024, 16000, 1, 0), (256, 256, 16000, 1, 0), (128, 128, 6400, 1, 0),
    (128, 512, 6400, 1, 0), (6400, 128, 128, 0, 0), (6400, 512, 128, 0, 1),
    ("conv", 6400, 128, 16, 128), ("conv", 6400, 2048, 3, 128), ("conv", 6400, 128, 8, 128),
]
PLANS = [(bm, bn, s) for bm, bn in ((128, 128), (128, 64), (64, 128), (64, 64))
         for s in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32)]


def timeit(f, reps=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    lib = _lib.load()
    for sh in SHAPES:
        if sh[0] == "conv":
            _, ML, Ci, taps, Co = sh
            x = torch.randn(32, ML // 32, Ci, device="cuda")
            W = torch.randn(taps, Ci, Co, device="cuda")
            out = torch.empty(32, ML // 32, Co, device="cuda")
            f = lambda: K.conv1d(x, W, out=out)   # noqa: E731
            M, N, Kd = ML, Co, Ci * taps
        else:
            M, N, Kd, at, bt = sh
            a = torch.randn(Kd, M, device="cuda").t() if at else torch.randn(M, Kd, device="cuda")
            b = torch.randn(N, Kd, device="cuda").t() if bt else torch.randn(Kd, N, device="cuda")
            c = torch.empty(M, N, device="cuda")
            f = lambda: K.gemm(a, b, c)   # noqa: E731
        fl = 2.0 * M * N * Kd
        lib.sat_gemm_force_plan(0, 0, 0)
        auto = timeit(f)
        res = []
        for bm, bn, s in PLANS:
            if s > 1 and Kd < 512:
                continue
            lib.sat_gemm_force_plan(bm, bn, s)
            try:
                us = timeit(f)
            except Exception:
                continue
            res.append((us, bm, bn, s))
        lib.sat_gemm_force_plan(0, 0, 0)
        res.sort()
        best = " ".join(f"{bm}x{bn}/s{s}:{us:.1f}" for us, bm, bn, s in res[:6])
        print(f"{str(sh):34s} auto {auto:7.1f} us {fl / auto / 1e6:6.1f} TF | best {best}", flush=True)


if __name__ == "__main__":
    main()
