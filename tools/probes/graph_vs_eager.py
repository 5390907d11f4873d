"""Where does a graphed training step first differ from the eager one?  Runs two identical
models (one GraphedStep, one eager Trainer.step) and compares forward outputs, gradients and
parameters after each step (diagnostic probe, not a test)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa
_sat_path.load()
import torch
from sat_amd import hparams, data, engine, train

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
cuda = torch.device("cuda:0")
hp = hparams.ljspeech_hparams()
b = data.synthetic_batch(hp, B, N=11, T=16, shape="ljs", seed=3)
batch = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
N, Tp = batch["source"].shape[1], batch["mel"].shape[1] // 2
m = engine.Tacotron(hp, cuda, seed=42)
tr = train.Trainer(m, B, N, Tp, seed=7)
m2 = engine.Tacotron(hp, cuda, seed=42)
tr2 = train.Trainer(m2, B, N, Tp, seed=7)


def cmp(tag):
    torch.cuda.synchronize()
    out = {"params": torch.equal(m.params, m2.params), "grads": torch.equal(m.grads, m2.grads),
           "loss": float(tr.last_loss[0]) == float(tr2.last_loss[0]),
           "masks": all(torch.equal(tr.masks[k], tr2.masks[k]) for k in tr.masks)}
    sv1, sv2 = tr.last_saved, tr2.last_saved
    d1, d2 = sv1["dec"].tensors, sv2["dec"].tensors
    for k in ("REC0", "S1", "AL1", "H2RAW", "G0", "ZH"):
        if k in d1 and d1[k] is not None:
            out[k] = torch.equal(d1[k], d2[k])
    bad = [k for k, v in out.items() if v is False]
    if not out["grads"]:
        g1, g2 = m.grads_dict(), m2.grads_dict()
        bad += [f"g:{k}" for k in g1 if not (g1[k] == g2[k]).all()]
    print(tag, "differs:", bad, flush=True)


g = train.GraphedStep(tr, batch, warmup=1)
tr2.step(batch)
print("after warmup: params equal", torch.equal(m.params, m2.params))
nosync = len(sys.argv) > 2
for i in range(6):
    g.replay()
    tr2.step(batch)
    if not nosync:
        cmp(f"replay {i}")
torch.cuda.synchronize()
cmp("end")
print("status graph", tr.status.tolist(), "health", m.health.tolist())
print("status eager", tr2.status.tolist(), "health", m2.health.tolist())
