"""Per-shape A/B of two tools/gemm_census.py outputs: python tools/census_diff.py A.txt B.txt"""
import sys


def load(f):
    d = {}
    for line in open(f):
        p = line.split()
        if len(p) == 14 and p[1].isdigit():
            d[tuple(p[:10])] = (int(p[10]), float(p[11]), float(p[12]))
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
rows = sorted(((a[k][0] * a[k][1], k) for k in a if k in b), reverse=True)
print(f"{'tag':18s} {'M':>6s} {'N':>6s} {'K':>6s} {'b':>4s} {'b2':>3s} am bm aK bN cnt   A_us   B_us  A_TF  B_TF")
for _, k in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 50]:
    x, y = a[k], b[k]
    print(f"{k[0][:18]:18s} {k[1]:>6s} {k[2]:>6s} {k[3]:>6s} {k[4]:>4s} {k[5]:>3s} {k[6]:>2s} {k[7]:>2s} "
          f"{k[8]:>2s} {k[9]:>2s} {x[0]:3d} {x[1]:6.1f} {y[1]:6.1f} {x[2]:5.1f} {y[2]:5.1f}")
