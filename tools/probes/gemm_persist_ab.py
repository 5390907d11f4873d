"""Persistent vs one-tile-per-workgroup grid of the LDS GEMM (EXPERIMENT, GPU):
    SAT_GEMM_PERSIST=1 python tools/probes/gemm_persist_ab.py > a.txt
    SAT_GEMM_PERSIST=0 python tools/probes/gemm_persist_ab.py > b.txt
Prints per step shape (tools/gemm_census.py, profiles/r05g_gemm_census.txt) the time (HIP
events, 20 launches after 3 warm-ups), TFLOP/s and a SHA-1 of the output bytes, so two runs
compare both speed and bit-identity."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import kernels as K  # noqa: E402

# (M, N, K, a_trans, b_trans, beta): A [M,K] (a_trans: stored [K,M]), B [K,N] (b_trans: [N,K])
SHAPES = [
    (16000, 1024, 256, 0, 1, 0.0), (16000, 1024, 544, 0, 1, 0.0), (16000, 544, 1024, 0, 0, 0.0),
    (16000, 1024, 128, 0, 1, 0.0), (16000, 256, 1024, 0, 0, 0.0), (16000, 256, 256, 0, 1, 0.0),
    (16000, 128, 1024, 0, 0, 0.0), (16000, 160, 256, 0, 1, 0.0), (6400, 512, 128, 0, 1, 0.0),
    (6400, 128, 256, 0, 0, 1.0), (256, 1024, 16000, 1, 0, 1.0), (544, 1024, 16000, 1, 0, 1.0),
    (288, 1024, 16000, 1, 0, 1.0), (128, 128, 6400, 1, 0, 1.0), (16000, 1024, 1024, 0, 1, 0.0),
]


def timeit(f, reps=20):
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
    g = torch.Generator(device="cuda").manual_seed(3)
    tag = os.environ.get("SAT_GEMM_PERSIST", "1")
    for M, N, Kd, at, bt, beta in SHAPES:
        a = torch.randn(*((Kd, M) if at else (M, Kd)), device="cuda", generator=g)
        b = torch.randn(*((N, Kd) if bt else (Kd, N)), device="cuda", generator=g)
        c0 = torch.randn(M, N, device="cuda", generator=g)
        A = a.t() if at else a
        B = b.t() if bt else b
        c = c0.clone()
        K.gemm(A, B, c, beta=beta)
        torch.cuda.synchronize()
        h = hashlib.sha1(c.cpu().numpy().tobytes()).hexdigest()[:12]
        us = timeit(lambda: K.gemm(A, B, c, beta=beta))
        print(f"persist={tag} {M}x{N}x{Kd} at={at} bt={bt} beta={beta}: {us:8.1f} us "
              f"{2.0 * M * N * Kd / us / 1e6:6.1f} TF/s  out {h}", flush=True)


if __name__ == "__main__":
    main()
