"""Attention-chain forward (dec_attn_fwd8_kernel) timing under probe switches
(SAT_FWD8_EXPT bits: 2 = no history stores, 4 = no poll sleep) and library variants, on the
training step's own buffers (B=32, N=200, T'=500).  Tools only: the switched runs' histories
are invalid.  Usage: python tools/probes/fwd8_expt.py [--save F] [--cmp F] [expt ...]
(--save writes the expt-0 histories, --cmp compares them with a file another library wrote)."""
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
ref = {k: kw[k].clone() for k in ("REC0", "C0", "H0RAW", "G0", "Q", "S1", "AL1", "S2", "ST",
                                  "LOC", "ZH") if kw.get(k) is not None}
names = ["wait B", "sync staged", "combine", "sync c", "c-dot+cell", "sync cell", "q part+pub A",
         "normalise", "loc+L", "wait A", "q sum", "energies", "sync+stats", "ctx+pub B", "h-dot"]


def run(expt, reps=6, prof=False):
    os.environ["SAT_FWD8_EXPT"] = str(expt)
    for _ in range(2):
        orig(**kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        orig(**kw)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    err = int(kw["err"][0].item())
    line = f"expt={expt}: {us:.1f} us/launch = {us / Tp:.3f} us/step (err {err})"
    if expt == 0:
        worst = max(float((kw[k] - ref[k]).abs().max()) for k in ref)
        line += f"  max|out-ref| {worst:.2e}"
    print(line, flush=True)
    if prof:
        pr = torch.zeros(256 * 16 + 8 * 8 * 16, dtype=torch.int64, device="cuda")
        orig(**dict(kw, prof=pr))
        torch.cuda.synchronize()
        pr = pr[:256 * 16].view(256, 16).cpu().double() / 100.0
        rows = [g + 32 * j for g in range(32) for j in range(8)]
        segs = [float(pr[rows, i].mean()) / Tp for i in range(15)]
        print("   " + "  ".join(f"{n} {v:.2f}" for n, v in zip(names, segs)) +
              f"  | total {sum(segs):.2f}", flush=True)
    os.environ.pop("SAT_FWD8_EXPT", None)


args = sys.argv[1:]
save = cmp = None
if "--save" in args:
    i = args.index("--save"); save = args[i + 1]; del args[i:i + 2]
if "--cmp" in args:
    i = args.index("--cmp"); cmp = args[i + 1]; del args[i:i + 2]
for e in [int(x) for x in args] or [0, 2, 4, 6]:
    run(e, prof=True)
run(0)
if save:
    torch.save({k: v.cpu() for k, v in ref.items()}, save)
if cmp:
    other = torch.load(cmp)
    for k in ref:
        d = (ref[k].cpu() - other[k]).abs()
        print(f"  vs {os.path.basename(cmp)}: {k:6s} max {float(d.max()):.3e} mean {float(d.mean()):.3e}")
