#!/usr/bin/env python3
"""Top-N kernel table from a rocprofv3 (ROCm 7.2) results database (rocpd SQLite, the default
output of `rocprofv3 --kernel-trace --stats -d DIR -o NAME`):

    python3 tools/rocpd_top.py gpurun_out/prof_r2/run_results.db "<command>" [N] [steps]

`steps` divides the totals into per-training-step milliseconds.  (top_kernels durations are in
microseconds in this schema: checked against the kernels view's ns start/end.)"""
import sqlite3
import sys


def main(path, cmd, n=30, steps=None):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels order by total_duration desc"))
    tot = sum(r[2] for r in rows)
    print(cmd)
    print(f"total kernel time {tot / 1e3:.1f} ms" +
          (f" over {steps} training steps = {tot / 1e3 / steps:.2f} ms/step" if steps else "") + "\n")
    hdr = f"{'kernel':72s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'share':>6s}"
    print(hdr + (f" {'ms/step':>8s}" if steps else ""))
    for name, calls, total, avg, pct in rows[:n]:
        nm = name.replace("sat::(anonymous namespace)::", "").replace("void ", "")[:72]
        line = f"{nm:72s} {calls:6d} {avg:9.2f} {total / 1e3:9.2f} {pct:5.1f}%"
        if steps:
            line += f" {total / 1e3 / steps:8.3f}"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 30,
         int(sys.argv[4]) if len(sys.argv) > 4 else None)
