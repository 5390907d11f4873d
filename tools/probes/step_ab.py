"""Step-time A/B of environment switches (tools only): runs ``bench.py`` (C2, hipGraph, no
baselines / extras) once per variant per round, interleaved, and prints ms/step and the loss.

Usage: python tools/probes/step_ab.py ROUNDS NAME=ENV[,ENV...] [NAME=...]
  e.g. python tools/probes/step_ab.py 2 base= late=SAT_DEC_WGRAD_FORK=pg
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
rounds = int(sys.argv[1])
variants = []
for a in sys.argv[2:]:
    name, _, envs = a.partition("=")
    env = dict(e.split("=", 1) for e in envs.split(",") if e)
    variants.append((name, env))
res = {n: [] for n, _ in variants}
for r in range(rounds):
    for name, env in variants:
        e = dict(os.environ, **env)
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20",
                            "--warmup", "5", "--no-cpu-baseline", "--no-extra", "--no-roofline"],
                           capture_output=True, text=True, env=e, cwd=ROOT, timeout=600)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not lines:
            print(f"{name}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
            sys.exit(1)
        d = json.loads(lines[-1])
        res[name].append((d["ms_per_step"], d["median_ms_per_step"], d["loss_last"]))
        print(f"round {r} {name:10s} {d['ms_per_step']:.3f} ms/step (median {d['median_ms_per_step']:.3f})"
              f" loss {d['loss_last']}", flush=True)
for name, v in res.items():
    print(f"{name:10s} " + " ".join(f"{x[0]:.3f}" for x in v))
