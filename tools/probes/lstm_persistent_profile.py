"""Segment clocks of the persistent decoder LSTM-stack kernels (tools only): per workgroup, the
wall-clock (100 MHz) time of each segment of one step over a full training step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

PROF = {}


def wrap(name):
    orig = getattr(K, name)

    def w(**kw):
        PROF[name] = torch.zeros(256 * 4, dtype=torch.int64, device="cuda")
        kw["prof"] = PROF[name]
        orig(**kw)
    setattr(K, name, w)


wrap("decoder_lstms_fwd")
wrap("decoder_lstms_bwd")
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=1)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
mk = {k: torch.tensor(v).cuda() for k, v in data.synthetic_masks(hp, B, 200, 500, seed=2).items()}
for _ in range(2):
    out, sv = m.forward(gb, mk, training=True)
    m.backward(sv)
torch.cuda.synchronize()
sv["dec"].tensors["attn_scratch"].check()
Tp = 501
SEGS = {"decoder_lstms_fwd": ["hand-off wait", "LDS staging", "dots + reduce", "cell + publish"],
        "decoder_lstms_bwd": ["barrier wait", "staging loads", "dots + reduce", "cells + stores"]}
for name in ("decoder_lstms_fwd", "decoder_lstms_bwd"):
    pr = PROF[name].view(256, 4).cpu().double() / 100.0   # us
    print(name)
    for i, n in enumerate(SEGS[name]):
        col = pr[:, i]
        print(f"  {n:22s} mean {col.mean() / Tp:6.2f} us/step  min {col.min() / Tp:6.2f}  "
              f"max {col.max() / Tp:6.2f}")
    print("  total us/step", float(pr.sum(1).mean() / Tp))
