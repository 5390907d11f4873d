"""MFMA-utilisation evidence for sat_gemm (north_star: "rocprof HBM GB/s and MFMA utilisation").

Drive one GEMM shape (GPU), for rocprofv3 PMC passes, one counter group per run:

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES ... GRBM_GUI_ACTIVE --kernel-trace \
        -d gpurun_out/pmc_gemm/<tag>_p1 -o pmc -- python3 tools/pmc_gemm.py run M N K [a_trans] [conv]

Summarise every pass directory of a tag into one JSON object:

    python3 tools/pmc_gemm.py summary gpurun_out/pmc_gemm <tag> M N K

MFMA pipe busy = SQ_VALU_MFMA_BUSY_CYCLES x 32 (sampling, below) / (1024 SIMDs x GRBM_GUI_ACTIVE);
achieved TF/s (and its fraction of the 157.3 TF/s f32 MFMA peak) from the kernel-trace durations
of the same dispatches.
"""
import glob
import json
import os
import re
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(M, N, Kd, at=0, conv=0, reps=30):
    sys.path.insert(0, ROOT)
    import _sat_path
    _sat_path.load()
    import torch
    from sat_amd import _lib, kernels as K
    plan = os.environ.get("SAT_GEMM_PLAN")   # "BM,BN,S": force the LDS kernel's plan
    if plan:
        _lib.load().sat_gemm_force_plan(*(int(x) for x in plan.split(",")))
    if conv:           # conv-bank-shaped Conv1D: x [32, M/32, N] (*) W [K/N taps, N, 128]
        S = 32
        x = torch.randn(S, M // S, N, device="cuda")
        W = torch.randn(Kd // N, N, 128, device="cuda")
        f = lambda: K.conv1d(x, W)   # noqa: E731
    else:
        a = torch.randn(Kd, M, device="cuda").t() if at else torch.randn(M, Kd, device="cuda")
        b = torch.randn(Kd, N, device="cuda")
        c = torch.empty(M, N, device="cuda")
        f = lambda: K.gemm(a, b, c)   # noqa: E731
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    print("ran", M, N, Kd, at, conv, reps)


def _rows(path):
    """(kernel name, counter name, value, duration ns) per dispatch from a rocpd database."""
    out = []
    for fn in glob.glob(f"{path}/**/*.db", recursive=True):
        db = sqlite3.connect(fn)
        tabs = [t for (t,) in db.execute("select name from sqlite_master where type='table'")]
        pmc = [t for t in tabs if "pmc_event" in t]
        ks = [t for t in tabs if "kernel_symbol" in t]
        kd = [t for t in tabs if "kernel_dispatch" in t]
        info = [t for t in tabs if "info_pmc" in t]
        if not (pmc and ks and kd and info):
            continue
        q = (f"select e.value, s.kernel_name, i.name, d.end - d.start, d.dispatch_id from {pmc[0]} e "
             f"join {kd[0]} d on e.event_id = d.event_id "
             f"join {ks[0]} s on d.kernel_id = s.id "
             f"join {info[0]} i on e.pmc_id = i.id")
        for v, kname, cname, dur, did in db.execute(q):
            out.append((kname, cname, float(v), float(dur), did))
    return out


def summary(base, tag, M, N, Kd, cus=256, xcds=8):
    acc, durs = {}, {}
    for d in sorted(glob.glob(os.path.join(base, f"{tag}_p*"))):
        for kname, cname, v, dur, did in _rows(d):
            if not re.search(r"gemm_(lds_)?kernel", kname):
                continue
            acc.setdefault(cname, []).append(v)
            durs.setdefault(d, {})[did] = dur
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    dur_ns = [x for dd in durs.values() for x in dd.values()]
    out = {"tag": tag, "M": M, "N": N, "K": Kd, "counters_avg_per_dispatch": avg}
    if dur_ns:
        t = sum(dur_ns) / len(dur_ns)
        out["avg_dispatch_us_profiled"] = round(t / 1e3, 2)
        out["tflops_profiled"] = round(2.0 * M * N * Kd / t / 1e3, 1)
    # The SQ block counters are collected from a 1/32 sample of the chip on this pool (SQ_WAVES
    # = launched waves / 32; SQ_VALU_MFMA_BUSY_CYCLES = 64 x MFMAs / 32 for the f32 32x32x2
    # MFMA): scale by `sample`.  GRBM_GUI_ACTIVE reads as cycles of one XCD.
    sample = 32
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        n_mfma = M * N * Kd / (32 * 32 * 2)
        out["mfma_busy_check"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] * sample / (64 * n_mfma), 3)
        if "GRBM_GUI_ACTIVE" in avg:
            out["mfma_pipe_busy_frac"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] * sample /
                                               (cus * 4 * avg["GRBM_GUI_ACTIVE"]), 4)
    if dur_ns:
        out["frac_of_f32_mfma_peak"] = round(out["tflops_profiled"] / 157.3, 4)
    if "SQ_WAVE_CYCLES" in avg:
        wc = avg["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in avg:
                out[k.lower() + "_frac"] = round(avg[k] / wc, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(*(int(x) for x in sys.argv[2:]))
    else:
        summary(sys.argv[2], sys.argv[3], *(int(x) for x in sys.argv[4:7]))
