#!/usr/bin/env python3
"""Top-N table of a rocprofv3 --stats kernel summary (CSV):

    python3 tools/stats_top.py gpurun_out/prof/run_kernel_stats.csv "<command>" [N]
"""
import csv
import sys


def main(path, cmd, n=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(cmd)
    print(f"total kernel time {tot / 1e6:.1f} ms\n")
    print(f"{'kernel':72s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'share':>6s}")
    for r in rows[:n]:
        name = r["Name"].replace("sat::(anonymous namespace)::", "").replace("void ", "")[:72]
        print(f"{name:72s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:9.2f} "
              f"{float(r['TotalDurationNs']) / 1e6:9.2f} {float(r['Percentage']):5.1f}%")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 30)
