"""``bench.py --gpus N`` as the driver runs it (no outer torchrun): the parent starts the N ranks
itself (torch.distributed.run child process, 127.0.0.1 rendezvous) and rank 0 prints ONE JSON
line.  Driven here on CPU under gloo with ``--plumbing`` (each rank times the per-step exchange
of the real arena instead of the GPU training step)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_launches_ranks_and_prints_one_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--plumbing", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 64 and d["steps"] == 2
    assert d["ms_per_step"] > 0
