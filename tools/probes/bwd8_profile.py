"""Attention-chain BPTT: one-utterance-per-8-workgroups kernel (decoder_persistent8_bwd.hip)
vs the 8 x 32 layout (SAT_ATTN_BWD8=0): HIP-event launch time on the training step's own
buffers, agreement of the outputs (dq compared as the sum over the old kernel's tile
partials), and the new kernel's segment clocks (tools only)."""
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
RD0 = kw["RD"].clone()                     # in: LSTM1's part (the call overwrites the c part)


def timed(flag, reps=3):
    os.environ["SAT_ATTN_BWD8"] = flag
    parts = 1 if flag == "1" else (int(kw["N"]) + 31) // 32
    dqp = torch.zeros(Tp, B, parts, 256, device="cuda")
    kk = dict(kw, DQP=dqp)
    times = []
    for i in range(reps + 1):
        kk["RD"].copy_(RD0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(**kk)
        e1.record()
        torch.cuda.synchronize()
        if i:
            times.append(e0.elapsed_time(e1) * 1e3)
    outs = {k: kk[k].clone() for k in ("DG0", "DE1", "DE2", "DFH", "RD")}
    outs["dq"] = dqp.sum(2)
    err = int(kk["err"][0].item())
    return sum(times) / len(times), outs, err


t_new, o_new, e_new = timed("1")
t_old, o_old, e_old = timed("0")
print(f"B={B} N=200 T'={Tp}: bwd8 {t_new:.1f} us/launch = {t_new / Tp:.2f} us/step (err {e_new}); "
      f"8x32 {t_old:.1f} us = {t_old / Tp:.2f} us/step (err {e_old})", flush=True)
for k in o_new:
    a, r = o_new[k], o_old[k]
    d = (a - r).abs()
    sc = float(r.abs().max()) or 1.0
    print(f"  {k:4s} max|new-old| {float(d.max()):.3e} (rel to max|old| {float(d.max()) / sc:.2e})")
os.environ["SAT_ATTN_BWD8"] = "1"
prof = torch.zeros(256 * 16, dtype=torch.int64, device="cuda")
kk = dict(kw, DQP=torch.zeros(Tp, B, 1, 256, device="cuda"), prof=prof)
kk["RD"].copy_(RD0)
orig(**kk)
torch.cuda.synchronize()
pr = prof.view(256, 16).cpu().double() / 100.0
names = ["Y: wait R/Q records", "Y: sync", "Y: dctx + DSN", "Y: sync", "Y: DA/DS2", "Y: scalars",
         "Y: sync", "Y: tanh backprop", "Y: sync", "Y: publish Q", "Z: wait Q", "Z: dq sum",
         "Z: unit reverse step", "Z: row-dot", "Z: sum + publish R"]
rows = [g + 32 * j for g in range(B) for j in range(8)]
for i, n in enumerate(names):
    col = pr[rows, i]
    print(f"  {n:24s} {float(col.mean()) / Tp:6.3f} us/step (max {float(col.max()) / Tp:6.3f})")
if float(pr[rows, 15].sum()) > 0:
    print(f"  {'  of which before prefetch':24s} {float(pr[rows, 15].mean()) / Tp:6.3f} us/step "
          "(slot 15; segment 2 is then the prefetch issue alone)")
print(f"  total {float(pr[rows].sum(1).mean()) / Tp:.3f} us/step")
