"""Segment clocks of the persistent decoder-attention kernel (tools only): per workgroup, the
wall-clock (100 MHz) time spent in phase A, barrier A, phase C, barrier C over a full decode."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

orig = K.decoder_attention_fwd
PROF = {}


def wrapped(**kw):
    PROF["buf"] = torch.zeros(256 * 8, dtype=torch.int64, device="cuda")
    kw["prof"] = PROF["buf"]
    orig(**kw)


K.decoder_attention_fwd = wrapped

hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=1)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
for _ in range(2):
    m.forward(gb, None, training=False, need_grad=False)
torch.cuda.synchronize()
pr = PROF["buf"].view(256, 8).cpu().double() / 100.0   # us
Tp = 500
names = ["phase A tail (query partial)", "barrier A", "phase C", "barrier C",
         "A: loads + combine", "A: tile normalise", "A: LSTM dot", "A: pointwise"]
for i, n in enumerate(names):
    col = pr[:, i]
    print(f"{n:28s} mean {col.mean() / Tp:7.2f} us/step  min {col.min() / Tp:7.2f}  "
          f"max {col.max() / Tp:7.2f}")
tile = pr[[g + 8 * j for g in range(8) for j in range(28)]]
print("tile WGs  phase C mean", float(tile[:, 2].mean() / Tp), "us/step")
