"""Attention-chain forward: one-utterance-per-8-workgroups kernel (decoder_persistent8.hip) vs
the 8 x 32 layout (SAT_ATTN_FWD8=0): HIP-event launch time on the training step's own buffers,
the new kernel's segment clocks, and bitwise agreement of the histories (tools only)."""
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
hp = hparams.ljspeech_hparams()
m = engine.Tacotron(hp, "cuda", seed=1)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape="max", seed=1)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
m.forward(gb, None, training=False, need_grad=True)
torch.cuda.synchronize()
kw = dict(KW)
Tp = int(kw["T"])


def timed(flag, reps=5):
    os.environ["SAT_ATTN_FWD8"] = flag
    for _ in range(2):
        orig(**kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        orig(**kw)
    e1.record()
    torch.cuda.synchronize()
    out = {k: kw[k].clone() for k in ("REC0", "C0", "H0RAW", "G0", "Q", "S1", "AL1", "S2", "ST",
                                      "LOC", "ZH") if kw.get(k) is not None}
    err = int(kw["err"][0].item())
    return e0.elapsed_time(e1) * 1e3 / reps, out, err


t_new, o_new, e_new = timed("1")
t_old, o_old, e_old = timed("0")
print(f"B={B} N=200 T'={Tp}: fwd8 {t_new:.1f} us/launch = {t_new / Tp:.2f} us/step (err {e_new}); "
      f"8x32 {t_old:.1f} us = {t_old / Tp:.2f} us/step (err {e_old})", flush=True)
for k in o_new:
    d = (o_new[k] - o_old[k]).abs()
    print(f"  {k:6s} max|new-old| {float(d.max()):.3e}  mean {float(d.mean()):.3e}")
os.environ["SAT_ATTN_FWD8"] = "1"
prof = torch.zeros(256 * 16 + 8 * 8 * 16 + 8 * 8 * 4 + 8 * 8 * 4 + 64, dtype=torch.int64,
                   device="cuda")
orig(**dict(kw, prof=prof))
torch.cuda.synchronize()
ev = prof[256 * 16:256 * 16 + 8 * 8 * 16].view(8, 8, 16).cpu().double() / 100.0   # [step][wave][event] us
sp = prof[256 * 16 + 8 * 8 * 16:256 * 16 + 8 * 8 * 20].view(8, 8, 4).cpu().double() / 100.0  # [step][wave][B drain, B poll, A drain, A poll] us
# (all zero unless libsat_hip was built with -DSAT_FWD8_TRACE=1)
ev = ev - ev[:, 0:1, 0:1]                                          # vs wave 0's loop start
print("per-wave event clocks of workgroup 1 (us after wave 0's step start, mean of steps 100..107)")
print("  wave " + " ".join(f"{k:6d}" for k in range(16)))
m = ev.mean(0)
for w in range(8):
    print(f"  {w:4d} " + " ".join(f"{float(m[w, k]):6.2f}" for k in range(16)))
for k, nm in enumerate(["B own-store drain", "B poll (after drain)", "A own-store drain",
                        "A poll (after drain)"]):
    print(f"  {nm:22s} us per wave: " + " ".join(f"{float(sp[:, w, k].mean()):.2f}" for w in range(8)))
pr = prof[:256 * 16].view(256, 16).cpu().double() / 100.0
names = ["wait B records", "sync (staged)", "combine + normalise", "sync (c)",
         "h+c dot + cell", "sync (cell)", "q partial + publish A", "-", "loc + L",
         "wait A records", "sync (A staged)", "q sum + energies", "sync (energies)", "stats",
         "ctx + publish B", "-"]
rows = [g + 32 * j for g in range(B) for j in range(8)]
for i, n in enumerate(names[:15]):
    col = pr[rows, i]
    print(f"  {n:24s} {float(col.mean()) / Tp:6.3f} us/step (max {float(col.max()) / Tp:6.3f})")
print(f"  total {float(pr[rows].sum(1).mean()) / Tp:.3f} us/step")
gv = prof[256 * 16 + 8 * 8 * 20:256 * 16 + 8 * 8 * 24].view(8, 8, 4).cpu().double()   # [step][j][ev]
if float(gv.abs().sum()) > 0:
    print("group 0 hand-off skew (trace build; us, relative to the earliest A publish of the step)")
    base = gv[:, :, 0].min(1, keepdim=True).values
    rel = (gv - base[:, :, None]) / 100.0
    m = rel[:7].mean(0)      # step 107's B staging lies past the recorded window
    for j in range(8):
        print(f"  wg {j}: A published {float(m[j, 0]):5.2f}  A staged {float(m[j, 1]):5.2f}  "
              f"B published {float(m[j, 2]):5.2f}  B staged {float(m[j, 3]):5.2f}")
# per tile column j (mean over the groups): which segment makes one workgroup of a group slower
print("segment clocks by workgroup j within the group (us/step, mean over groups)")
print("  " + " ".join(f"{n[:10]:>10s}" for n in names[:15] if n != "-"))
for jj in range(8):
    rj = [g + 32 * jj for g in range(B)]
    print(f"  j={jj} " + " ".join(f"{float(pr[rj, i].mean()) / Tp:10.3f}"
                                  for i, n in enumerate(names[:15]) if n != "-"))
