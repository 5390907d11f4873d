"""Debug aid (GPU): persistent decoder path vs the per-step launch path on one small case;
prints, per history tensor, the max |diff| and the first decoder step where it exceeds 1e-5."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams, params  # noqa: E402

B, N, T = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (8, 40, 24)))
hp = hparams.ljspeech_hparams()
vals = params.init_params(hp, seed=5)
b = data.synthetic_batch(hp, B, N=N, T=T, shape="ljs", seed=3)
Np, Tp = b["source"].shape[1], b["mel"].shape[1] // hp.outputs_per_step
mk = data.synthetic_masks(hp, B, Np, Tp, seed=4)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
gm = {k: torch.tensor(v).cuda() for k, v in mk.items()}
svs = []
for persistent in (False, True):
    m = engine.Tacotron(hp, "cuda", init_values=vals, persistent_decoder=persistent)
    out, sv = m.forward(gb, gm, training=True)
    torch.cuda.synchronize()
    if persistent:
        sv["dec"].tensors["attn_scratch"].check()
    svs.append(sv["dec"].tensors)
r, a = svs
print("lengths", b["source_length"] if "source_length" in b else "")
for name in ("REC0", "C0", "H0RAW", "G0", "Q", "S1", "AL1", "S2", "ST", "LOC"):
    x, y = a[name].float(), r[name].float()
    d = (x - y).abs()
    steps = d.reshape(d.shape[0], -1).amax(1)
    bad = (steps > 1e-5).nonzero()
    first = int(bad[0]) if len(bad) else -1
    print(f"{name:6s} shape {tuple(d.shape)} max {float(d.max()):.3e} first step {first}")
    if first >= 0:
        row = d[first].reshape(B, -1)
        bb = int(row.amax(1).argmax())
        cols = (row[bb] > 1e-5).nonzero().flatten()[:12].tolist()
        print(f"        utt {bb} cols {cols}")
        print("        got ", x[first].reshape(B, -1)[bb, cols[:6]].tolist())
        print("        want", y[first].reshape(B, -1)[bb, cols[:6]].tolist())
