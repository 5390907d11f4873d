"""Stage-by-stage check of the CBHG backward at a given batch (tools only): records the inputs and
outputs of sat_conv1d dX (proj2 / proj1), sat_maxpool2_bwd and sat_bn_bwd inside one training
step and recomputes each in float64 torch on the GPU from the recorded inputs, so a discrepancy
is pinned to the stage that makes it (per 128-channel block for the 2048-wide bank).

Usage: python tools/probes/enc_bwd_stages.py [B] [shape] [seed]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams, params  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
shape = sys.argv[2] if len(sys.argv) > 2 else "max"
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 51
REC = []


def wrap(name, fn, outs):
    def w(*a, **kw):
        r = fn(*a, **kw)
        torch.cuda.synchronize()
        REC.append((name, [x.clone() if isinstance(x, torch.Tensor) else x for x in a],
                    {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in kw.items()},
                    r.clone() if isinstance(r, torch.Tensor) else None))
        return r
    return w


K.maxpool2_bwd = wrap("maxpool2_bwd", K.maxpool2_bwd, None)
K.conv1d_dx = wrap("conv1d_dx", K.conv1d_dx, None)
K.bn_bwd = wrap("bn_bwd", K.bn_bwd, None)

hp = hparams.ljspeech_hparams()
vals = params.init_params(hp, seed=5)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape=shape, seed=seed)
Np, Tp = b["source"].shape[1], b["mel"].shape[1] // hp.outputs_per_step
mk = data.synthetic_masks(hp, B, Np, Tp, seed=seed + 1)
m = engine.Tacotron(hp, "cuda", init_values=vals)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
gm = {k: torch.tensor(v).cuda() for k, v in mk.items()}
out, sv = m.forward(gb, gm, training=True)
m.backward(sv)
torch.cuda.synchronize()


def rel(a, r):
    return float((a.double() - r).abs().max() / r.abs().max().clamp_min(1e-30))


for name, a, kw, r in REC:
    if name == "maxpool2_bwd":
        x, dy, dx = a[0].double(), a[1].double(), a[2].double()
        nxt = torch.cat([x[:, 1:], x[:, -1:]], 1)
        first = x >= nxt                                 # window [n, n+1]: the max's first index
        g = torch.where(first, dy, torch.zeros_like(dy))
        prv = torch.cat([x[:, :1], x[:, :-1]], 1)
        take = torch.zeros_like(x, dtype=torch.bool)
        take[:, 1:] = prv[:, 1:] < x[:, 1:]
        g[:, 1:] += torch.where(take[:, 1:], dy[:, :-1], torch.zeros_like(dy[:, 1:]))
        ties = int(((x[:, :-1] == x[:, 1:]) & (x[:, :-1] > 0)).sum())
        ties0 = int(((x[:, :-1] == x[:, 1:]) & (x[:, :-1] == 0)).sum())
        C = x.shape[-1]
        per = [rel(dx[..., i:i + 128], g[..., i:i + 128]) for i in range(0, C, 128)]
        print(f"maxpool2_bwd {tuple(x.shape)}: rel err {rel(dx, g):.3e}; positive ties {ties}, "
              f"zero ties {ties0}; per 128-channel block: " + " ".join(f"{e:.1e}" for e in per),
              flush=True)
    elif name == "conv1d_dx":
        dy, W = a[0].double(), a[1].double()
        taps, Ci, Co = W.shape
        pl = (taps - 1) // 2
        # y[n] = sum_j x[n + j - pl] W[j]  =>  dx[m] = sum_j dy[m - j + pl] W[j]^T
        N = dy.shape[1]
        dyp = torch.nn.functional.pad(dy, (0, 0, taps - 1 - pl, pl))
        ref = sum(dyp[:, taps - 1 - j:taps - 1 - j + N] @ W[j].t() for j in range(taps))
        got = (r if r is not None else kw.get("out")).double()
        per = [rel(got[..., i:i + 128], ref[..., i:i + 128]) for i in range(0, ref.shape[-1], 128)]
        print(f"conv1d_dx dy {tuple(dy.shape)} W {tuple(W.shape)}: rel err {rel(got, ref):.3e}; "
              f"per 128-col block max {max(per):.1e} at {per.index(max(per))}", flush=True)
    elif name == "bn_bwd":
        dy, x, y, dx = a[0].double(), a[1].double(), a[2], a[3].double()
        mean, var, gamma = a[4].double(), a[5].double(), a[6].double()
        g_dy = dy if y is None else dy * (y.double() > 0)
        xh = (x - mean) / torch.sqrt(var + 1e-3)
        Mr = x.shape[0]
        dbeta = g_dy.sum(0)
        dgamma = (g_dy * xh).sum(0)
        ref = gamma / torch.sqrt(var + 1e-3) * (g_dy - dbeta / Mr - xh * dgamma / Mr)
        C = x.shape[1]
        per = [rel(dx[:, i:i + 128], ref[:, i:i + 128]) for i in range(0, C, 128)]
        print(f"bn_bwd {tuple(x.shape)}: dx rel err {rel(dx, ref):.3e}; per 128-channel block: "
              + " ".join(f"{e:.1e}" for e in per), flush=True)
