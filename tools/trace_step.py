#!/usr/bin/env python3
"""Per-kernel time of ONE replayed training step from a rocprofv3 kernel trace (CSV):

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o tr -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline
    python3 tools/trace_step.py gpurun_out/trace/.../tr_kernel_trace.csv

Steps are delimited by the first mask-RNG launch of each step (rng_fill_kernel after a gap of
non-RNG kernels); the LAST complete step is summarised: span, busy time, dispatch count, and
per kernel the count / total / average device time and the average gap before it."""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in rows)
    starts = [i for i, e in enumerate(ev)
              if "rng_fill" in e[2] and (i == 0 or "rng_fill" not in ev[i - 1][2])]
    if len(starts) < 2:
        raise SystemExit("need >= 2 steps in the trace")
    a, b = starts[-2], starts[-1]
    # the last step runs to the end of the trace; the one before is complete for sure
    seg = ev[a:b]
    span = seg[-1][1] - seg[0][0]
    busy = sum(e - s for s, e, _ in seg)
    stats = defaultdict(lambda: [0, 0, 0])
    for i, (s, e, n) in enumerate(seg):
        k = n.replace("sat::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        st = stats[k]
        st[0] += 1
        st[1] += e - s
        st[2] += (s - seg[i - 1][1]) if i else 0
    print(f"step: {len(seg)} dispatches, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, "
          f"gaps {(span - busy) / 1e6:.3f} ms")
    print(f"{'kernel':60s} {'n':>6s} {'total_ms':>9s} {'avg_us':>8s} {'gap_us':>7s} {'share':>6s}")
    for k, (c, t, g) in sorted(stats.items(), key=lambda kv: -kv[1][1] - kv[1][2]):
        print(f"{k:60s} {c:6d} {t / 1e6:9.3f} {t / c / 1e3:8.2f} {g / c / 1e3:7.2f} "
              f"{(t + g) / span:6.1%}")


if __name__ == "__main__":
    main(sys.argv[1])
