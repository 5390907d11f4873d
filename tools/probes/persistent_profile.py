"""Segment clocks of the persistent decoder-attention kernel (tools only): per workgroup, the
wall-clock (100 MHz) time spent in each segment of a step (poll waits, combine, LSTM dot,
cell + publish, normalise, tile) over a full decode."""
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
    PROF["buf"] = torch.zeros(256 * 16 + 500 * 256 * 8, dtype=torch.int64, device="cuda")
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
pr = PROF["buf"][:256 * 16].view(256, 16).cpu().double() / 100.0   # us
Tp = 500
names = ["A: poll partials + h", "A: combine", "A: LSTM dot + reduce", "A: publish (after sync)",
         "A: tile normalise", "C: poll query partials", "C: energies", "C: (unused)",
         "C: stats", "C: contexts", "C: publish", "C: tanh/loc stores", "A: cell + stores",
         "A: sync after cell", "C: q reduce", "(unused)"]
for i, n in enumerate(names):
    col = pr[:, i]
    print(f"{n:28s} mean {col.mean() / Tp:7.2f} us/step  min {col.min() / Tp:7.2f}  "
          f"max {col.max() / Tp:7.2f}")
print(f"total us/step {float(pr.sum(1).mean()) / Tp:.2f}")
tile = pr[[g + 8 * j for g in range(8) for j in range(28)]]
print("tile WGs:", " ".join(f"{float(tile[:, i].mean() / Tp):.2f}" for i in range(16)))

# hand-off latencies from the event trace (utterance 0 of each group, steps 50..449)
tr = PROF["buf"][256 * 16:].view(500, 256, 8).cpu().double() / 100.0   # us
ntiles = 7
import statistics as st
rows = {k: [] for k in ("p_all", "p_tile", "p_non", "p_light", "p_start", "q", "q_light", "q_start",
                        "skew_p", "skew_q")}
for g in range(8):
    tiles = [g + 8 * j for j in range(ntiles)]          # tiles of utterance 0 (ub = 0)
    non = [g + 8 * j for j in range(28, 32)]
    allw = [g + 8 * j for j in range(32)]
    for t in range(50, 450):
        last = tr[t, tiles, 3].max()
        rows["skew_p"].append(float(last - tr[t, tiles, 3].min()))
        rows["p_all"].append(float(tr[t + 1, allw, 0].mean() - last))
        rows["p_tile"].append(float(tr[t + 1, tiles, 0].mean() - last))
        rows["p_non"].append(float(tr[t + 1, non, 0].mean() - last))
        lt = tr[t + 1, allw, 4]
        lt = lt[lt > 0]
        if len(lt):
            rows["p_light"].append(float(lt.mean() - last))
        rows["p_start"].append(float(tr[t + 1, tiles, 6].mean() - last))
        qlast = tr[t, allw, 1].max()
        rows["skew_q"].append(float(qlast - tr[t, allw, 1].min()))
        rows["q"].append(float(tr[t, tiles, 2].mean() - qlast))
        ql = tr[t, tiles, 5]
        ql = ql[ql > 0]
        if len(ql):
            rows["q_light"].append(float(ql.mean() - qlast))
        rows["q_start"].append(float(tr[t, tiles, 7].mean() - qlast))
for k, v in rows.items():
    print(f"{k:8s} mean {st.mean(v):6.2f} us  (n={len(v)})")
print("p_*: vs the last tile record publish of utterance 0; q_*: vs the last query-partial publish")
