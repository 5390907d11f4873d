"""Time every GEMM launch of one training step in isolation (GPU).

    python tools/gemm_census.py [--batch 32] [--top 40]

Runs one eager step with kernels.GEMM_LOG enabled, then replays each recorded descriptor 10x
between HIP events and prints shape, time and achieved TFLOP/s, grouped by identical shape.
"""
import argparse
import collections
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import _lib, data, engine, hparams, train  # noqa: E402
from sat_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--sweep", type=int, default=0,
                    help="also time every forced LDS-kernel plan on the N costliest shapes")
    a = ap.parse_args()
    hp = hparams.ljspeech_hparams()
    m = engine.Tacotron(hp, "cuda")
    b = data.synthetic_batch(hp, a.batch, N=200, T=1000, shape="max", seed=1)
    batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
    tr = train.Trainer(m, a.batch, 200, 500)
    tr.step(batch)
    torch.cuda.synchronize()
    K.GEMM_LOG = []
    tr.step(batch)
    torch.cuda.synchronize()
    log, K.GEMM_LOG = K.GEMM_LOG, None
    lib = _lib.load()
    groups = collections.OrderedDict()
    descs = {}
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sites = collections.defaultdict(collections.Counter)
    for tag, d, site in log:
        key = (tag, d.M, d.N, d.K, d.batch, d.batch2, d.a_mode, d.b_mode, d.a_sk == 1, d.b_sn == 1)
        sites[key][site] += 1
        if key not in groups:
            descs[key] = d
            for _ in range(2):
                lib.sat_gemm(ctypes.byref(d), ctypes.c_void_p(s.cuda_stream))
            e0.record()
            for _ in range(10):
                lib.sat_gemm(ctypes.byref(d), ctypes.c_void_p(s.cuda_stream))
            e1.record()
            torch.cuda.synchronize()
            groups[key] = [0, e0.elapsed_time(e1) / 10 * 1e3]
        groups[key][0] += 1
    rows = []
    for key, (cnt, us) in groups.items():
        tag, M, N, Kd, nb, nb2, am, bm, ak, bn = key
        fl = 2.0 * M * N * Kd * max(nb, 1) * max(nb2, 1)
        rows.append((cnt * us, cnt, us, fl / us / 1e6, key))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"{len(log)} gemm launches, {len(rows)} shapes, isolated total {tot / 1e3:.2f} ms")
    print(f"{'tag':22s} {'M':>6s} {'N':>6s} {'K':>6s} {'b':>4s} {'b2':>3s} am bm aK bN  cnt   us/launch  TFLOP/s  total_ms")
    for tot_us, cnt, us, tf, key in rows[:a.top]:
        tag, M, N, Kd, nb, nb2, am, bm, ak, bn = key
        print(f"{tag:22s} {M:6d} {N:6d} {Kd:6d} {nb:4d} {nb2:3d} {am:2d} {bm:2d} {int(ak):2d} {int(bn):2d} "
              f"{cnt:4d} {us:10.1f} {tf:8.1f} {tot_us / 1e3:8.3f}  "
              + ", ".join(f"{k}x{v}" for k, v in sites[key].most_common(3)))
    if a.sweep:
        sweep(lib, descs, [r[4] for r in rows[:a.sweep]])



def sweep(lib, descs, keys):
    """Forced (BM, BN, S) plans of the LDS kernel on the step's own descriptors."""
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for key in keys:
        d = descs[key]
        res = []
        for bm, bn in ((256, 128), (128, 256), (128, 128), (128, 64), (64, 128), (64, 64)):
            for sp in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32):
                if sp > 1 and d.K < 512:
                    continue
                lib.sat_gemm_force_plan(bm, bn, sp)
                for _ in range(2):
                    lib.sat_gemm(ctypes.byref(d), ctypes.c_void_p(s.cuda_stream))
                e0.record()
                for _ in range(10):
                    lib.sat_gemm(ctypes.byref(d), ctypes.c_void_p(s.cuda_stream))
                e1.record()
                torch.cuda.synchronize()
                res.append((e0.elapsed_time(e1) / 10 * 1e3, bm, bn, sp))
        lib.sat_gemm_force_plan(0, 0, 0)
        res.sort()
        print(key[:6], " ".join(f"{bm}x{bn}/s{sp}:{us:.1f}" for us, bm, bn, sp in res[:5]), flush=True)


if __name__ == "__main__":
    main()
