"""A/B of the attention-chain forward's schedules on one box (tools only): the training step's
own sat_decoder_attention_fwd launch (B=32, N=200, T'=500) timed with HIP events under
SAT_FWD8_RED=1 (records reduced at staging) and =0 (two-barrier staging), interleaved, plus the
largest history difference between the two (they differ only in summation order).

Usage: python tools/probes/fwd8_ab.py [B] [rounds]
"""
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
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=1)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
m.forward(gb, None, training=False, need_grad=True)
torch.cuda.synchronize()
kw = dict(KW)
Tp = int(kw["T"])
HIST = ("REC0", "C0", "H0RAW", "G0", "Q", "S1", "AL1", "S2", "ST", "LOC", "ZH")


def timed(flag, reps=5):
    os.environ["SAT_FWD8_RED"] = flag
    orig(**kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        orig(**kw)
    e1.record()
    torch.cuda.synchronize()
    assert int(kw["err"][0].item()) == 0
    return e0.elapsed_time(e1) * 1e3 / reps


res = {"1": [], "0": []}
for r in range(rounds):
    for flag in ("1", "0"):
        res[flag].append(timed(flag))
for flag, name in (("0", "two-barrier staging"), ("1", "reduced at staging")):
    v = sorted(res[flag])
    print(f"B={B} T'={Tp} {name:22s}: {' '.join(f'{x:7.1f}' for x in res[flag])} us/launch "
          f"-> median {v[len(v) // 2] / Tp:.3f} us/step", flush=True)
outs = {}
for flag in ("0", "1"):
    os.environ["SAT_FWD8_RED"] = flag
    orig(**kw)
    torch.cuda.synchronize()
    outs[flag] = {k: kw[k].clone() for k in HIST if kw.get(k) is not None}
for k in outs["0"]:
    d = (outs["1"][k] - outs["0"][k]).abs()
    print(f"  {k:6s} max|red - two| {float(d.max()):.3e}  mean {float(d.mean()):.3e}")
