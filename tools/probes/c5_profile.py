"""C5 free-running decode (bench.py c5_free_running) on its own, for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace --stats -d DIR -o c5 -- python3 tools/probes/c5_profile.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams  # noqa: E402
from sat_amd.inference import FreeRunningDecoder  # noqa: E402

B, steps = 8, 500
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1234)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=55)
batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
dec = FreeRunningDecoder(m, max_iters=steps, min_iters=steps, check_every=25, graphs=True)
dec.run(batch)
torch.cuda.synchronize()
t0 = time.perf_counter()
dec.run(batch)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"C5: {dt * 1e3:.1f} ms per decode = {dt * 1e6 / steps:.1f} us per decoder step", flush=True)
