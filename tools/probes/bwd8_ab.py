"""A/B of the attention-chain BPTT's Q staging on one box (tools only): the training step's own
sat_decoder_attention_bwd launch (B=32, N=200, T'=500, train mode) timed with HIP events under
SAT_BWD8_RED=1 (records reduced at staging) and =0 (stage, barrier, serial sum, barrier),
interleaved, plus the largest output difference (summation order only).

Usage: python tools/probes/bwd8_ab.py [B] [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

orig = K.decoder_attention_bwd
KW = {}


def rec(**kw):
    KW.update(kw)
    orig(**kw)


K.decoder_attention_bwd = rec
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=1)
mk = data.synthetic_masks(hp, B, 200, 500, seed=2)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
gm = {k: torch.tensor(v).cuda() for k, v in mk.items()}
out, sv = m.forward(gb, gm, training=True)
m.backward(sv)
torch.cuda.synchronize()
kw = dict(KW)
Tp = int(kw["T"])
RD0 = kw["RD"].clone()          # in: LSTM1's part (the call overwrites the c part)


def run(flag):
    os.environ["SAT_BWD8_RED"] = flag
    kw["RD"].copy_(RD0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    orig(**kw)
    e1.record()
    torch.cuda.synchronize()
    assert int(kw["err"][0].item()) == 0
    return e0.elapsed_time(e1) * 1e3


res = {"1": [], "0": []}
for flag in ("1", "0"):
    run(flag)
for r in range(rounds):
    for flag in ("1", "0"):
        res[flag].append(sum(run(flag) for _ in range(3)) / 3)
for flag, name in (("0", "two-barrier Q staging"), ("1", "Q reduced at staging")):
    v = sorted(res[flag])
    print(f"B={B} T'={Tp} {name:22s}: {' '.join(f'{x:7.1f}' for x in res[flag])} us/launch "
          f"-> median {v[len(v) // 2] / Tp:.3f} us/step", flush=True)
outs = {}
for flag in ("0", "1"):
    run(flag)
    outs[flag] = {k: kw[k].clone() for k in ("DG0", "DE1", "DE2", "DFH", "RD", "DQP")}
for k in outs["0"]:
    d = (outs["1"][k] - outs["0"][k]).abs()
    print(f"  {k:4s} max|red - two| {float(d.max()):.3e}  mean {float(d.mean()):.3e}")
