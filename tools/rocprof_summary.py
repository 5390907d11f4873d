#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite (.db) kernel trace: per-kernel count / total / avg / share, and the
busy-vs-wall ratio of the dispatch stream (gaps between kernels = launch boundaries)."""
import sqlite3
import sys
from collections import defaultdict


def main(path, last=None):
    db = sqlite3.connect(path)
    rows = db.execute(
        "select k.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol k on d.kernel_id = k.id order by d.start").fetchall()
    if last:
        rows = rows[-last:]
    stats = defaultdict(lambda: [0, 0])
    for name, s, e in rows:
        short = name.split("(")[0].replace("void ", "")[:70]
        stats[short][0] += 1
        stats[short][1] += e - s
    busy = sum(v[1] for v in stats.values())
    wall = rows[-1][2] - rows[0][1] if rows else 0
    print(f"dispatches {len(rows)}  busy {busy/1e6:.3f} ms  span {wall/1e6:.3f} ms  "
          f"busy/span {busy/max(wall,1):.3f}")
    print(f"{'kernel':70s} {'count':>7s} {'total_ms':>10s} {'avg_us':>9s} {'share':>6s}")
    for k, (c, t) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:70s} {c:7d} {t/1e6:10.3f} {t/c/1e3:9.3f} {t/max(busy,1):6.1%}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
