"""Where a one-launch C5 decode's wall time goes (host-synchronised sections, second run)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams  # noqa: E402
from sat_amd import kernels as K  # noqa: E402
from sat_amd.inference import FreeRunningDecoder  # noqa: E402
from sat_amd.model import encoder_fwd  # noqa: E402

B, steps = 8, 500
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1234)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=55)
batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
dec = FreeRunningDecoder(m, max_iters=steps, min_iters=steps, check_every=25, graphs=True)
dec.run(batch)
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    dec.run(batch)
    torch.cuda.synchronize()
    print(f"run(): {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
pl = dec._plans[(B, 200, steps)]
P, d = m.P, m.d


def sect(name, fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: {1e3 * (time.perf_counter() - t0) / n:.3f} ms", flush=True)


sect("encoder_fwd", lambda: encoder_fwd(P, m.bn, hp, d, batch["source"], batch["source_length"],
                                         None, False, m.ws, {}))
sect("_prepare", lambda: dec._prepare(pl, batch, None))
sect("_pack_persistent", lambda: dec._pack_persistent(pl))
sect("_run_persistent", lambda: dec._run_persistent(pl, steps), n=3)
