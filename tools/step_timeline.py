"""One training step's kernel timeline from a rocprofv3 kernel trace (CPU tool).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o tr -- python3 bench.py --steps 3 ...
    python tools/step_timeline.py OUT/tr_kernel_trace.csv [--list]

The step is the interval between the last two Adam launches.  With the second stream
(backward.Aux, model.model_forward) kernels overlap, so summed kernel durations exceed the wall
time; this reports what the wall time is made of instead:
  * union busy time (some kernel running) and the idle gaps;
  * per kernel class (persistent recurrences, GEMM, other): the summed durations, the time at
    least one kernel of the class runs, and the time it runs ALONE (no other class beside it) --
    the part of the step only that class can shorten.
"""
import csv
import re
import sys

PERSISTENT = ("dec_attn_fwd8", "dec_attn_bwd8", "dec_lstm_fwd", "dec_lstm_bwd", "enc_lstm_fwd",
              "enc_lstm_bwd", "attn_param_grad")


def kclass(name):
    if any(p in name for p in PERSISTENT):
        return "recurrence"
    if "gemm" in name:
        return "gemm"
    return "other"


def short(name):
    name = name.replace("void ", "").replace("sat::(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name.replace("sat::", ""))[:60]


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def subtract(a, b):
    """intervals of a not covered by b (both unions)"""
    out = []
    j = 0
    for s, e in a:
        cur = s
        while j < len(b) and b[j][1] <= cur:
            j += 1
        k = j
        while k < len(b) and b[k][0] < e:
            if b[k][0] > cur:
                out.append([cur, b[k][0]])
            cur = max(cur, b[k][1])
            k += 1
        if cur < e:
            out.append([cur, e])
    return out


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    adam = [r for r in rows if "adam_update" in r["Kernel_Name"]]
    if len(adam) < 2:
        sys.exit("need at least two steps in the trace")
    t0, t1 = adam[-2]["e"], adam[-1]["e"]
    step = [r for r in rows if r["s"] >= t0 and r["e"] <= t1]
    wall = t1 - t0
    allu = union([(r["s"], r["e"]) for r in step])
    print(f"step wall {wall / 1e6:.3f} ms, {len(step)} kernels, union busy {length(allu) / 1e6:.3f} ms"
          f" (idle {(wall - length(allu)) / 1e6:.3f} ms)")
    classes = {}
    for r in step:
        classes.setdefault(kclass(r["Kernel_Name"]), []).append(r)
    unions = {c: union([(r["s"], r["e"]) for r in v]) for c, v in classes.items()}
    print(f"{'class':12s} {'launches':>8s} {'sum of durations':>17s} {'running':>9s} {'alone':>9s}  (ms)")
    for c in ("recurrence", "gemm", "other"):
        if c not in classes:
            continue
        others = union([iv for k, u in unions.items() if k != c for iv in u])
        alone = subtract(unions[c], others)
        print(f"{c:12s} {len(classes[c]):8d} {sum(r['e'] - r['s'] for r in classes[c]) / 1e6:17.3f}"
              f" {length(unions[c]) / 1e6:9.3f} {length(alone) / 1e6:9.3f}")
    if "--list" in sys.argv:
        for r in step:
            print(f"{(r['s'] - t0) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f} q{r['Queue_Id']} "
                  f"{short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
