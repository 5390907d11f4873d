"""A/B of the attention-chain forward (decoder_persistent8.hip) with and without the energy-tanh
history ZH (3.3 GB per launch at C2): HIP-event launch time on the step's own buffers."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

orig = K.decoder_attention_fwd
KW = {}


def rec(**kw):
    KW.update(kw)
    orig(**kw)


K.decoder_attention_fwd = rec
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1)
b = data.synthetic_batch(hp, 32, N=200, T=1000, shape="max", seed=1)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
m.forward(gb, None, training=False, need_grad=True)
torch.cuda.synchronize()
kw = dict(KW)
Tp = int(kw["T"])


def timed(kw, reps=5):
    for _ in range(2):
        orig(**kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        orig(**kw)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for name, k in (("with ZH", kw), ("no ZH", dict(kw, ZH=None)), ("no ZH, no LOC", dict(kw, ZH=None, LOC=None))):
    t = timed(k)
    print(f"{name:16s} {t:8.1f} us/launch = {t / Tp:.3f} us/step", flush=True)
