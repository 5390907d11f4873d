"""How many piecewise-linear decisions of the CBHG forward differ between the fp32 HIP step and
the float64 oracle at a given batch (tools only): the conv-bank ReLU gates (per 128-channel
block = one conv width K1..K16) and the max-pool window choices.  A flipped gate routes a whole
element's gradient differently, so parameter gradients upstream of it can differ by far more
than fp32 rounding while every kernel is exact on its own inputs.

Usage: python tools/probes/enc_kinks.py [B] [shape] [seed]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from oracle import sat_oracle as O  # noqa: E402
from sat_amd import data, engine, hparams, params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
shape = sys.argv[2] if len(sys.argv) > 2 else "max"
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 51
hp = hparams.ljspeech_hparams()
vals = params.init_params(hp, seed=5)
b = data.synthetic_batch(hp, B, N=200, T=1000, shape=shape, seed=seed)
Np, Tp = b["source"].shape[1], b["mel"].shape[1] // hp.outputs_per_step
mk = data.synthetic_masks(hp, B, Np, Tp, seed=seed + 1)
m = engine.Tacotron(hp, "cuda", init_values=vals)
gb = {k: torch.tensor(v).cuda() for k, v in b.items()}
gm = {k: torch.tensor(v).cuda() for k, v in mk.items()}
out, sv = m.forward(gb, gm, training=True)
torch.cuda.synchronize()
bank_gpu = sv["bank"].double().cpu()                       # relu(BN(conv)) [B, N, 2048]

p = O.to_torch(vals)
bufs = O.to_torch(params.init_bn_buffers(hp))
masks = O.to_torch(mk)
x = p["embedding"][O.to_torch(b)["source"]]
for i in range(len(hp.encoder_prenet_out_units)):
    x = O.prenet(x, p, f"encoder/prenet{i}", masks[f"enc/prenet{i}"])
z = torch.cat([O.conv_bn(x, p, bufs, f"encoder/cbhg/conv_bank/K{k}", True, relu=False)
               for k in range(1, hp.max_filter_width + 1)], dim=-1)   # pre-ReLU, float64
gate64, gate32 = z > 0, bank_gpu > 0
flips = (gate64 != gate32)
mp64 = z.clamp_min(0)
nxt = torch.cat([mp64[:, 1:], mp64[:, -1:]], 1)
first64 = mp64 >= nxt
nxt32 = torch.cat([bank_gpu[:, 1:], bank_gpu[:, -1:]], 1)
first32 = bank_gpu >= nxt32
pool = (first64 != first32) & ((mp64 > 0) | (nxt > 0))
print(f"B={B} {shape}: bank elements {z.numel()}, |BN out| min over flipped gates "
      f"{float(z[flips].abs().min()) if flips.any() else float('nan'):.2e}")
print("  per conv width: gate flips / max-pool choice flips")
for k in range(hp.max_filter_width):
    sl = slice(128 * k, 128 * (k + 1))
    print(f"    K{k + 1:2d}: {int(flips[..., sl].sum()):5d} / {int(pool[..., sl].sum()):5d}")
print(f"  max |bank fp32 - fp64| {float((bank_gpu - z.clamp_min(0)).abs().max()):.3e}")
