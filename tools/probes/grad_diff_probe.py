"""Which parameter gradients differ between two configurations of the same step (tools only):
runs tests/test_model_bwd_gpu.py's small eval step (B=3, N=17, T=24) in this process and prints,
per parameter, the max difference against the float64 oracle.  Usage: python grad_diff_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sat_amd import data, engine, hparams, params  # noqa: E402
from oracle import sat_oracle as O  # noqa: E402

hp = hparams.ljspeech_hparams()
vals = params.init_params(hp, seed=5)
m = engine.Tacotron(hp, "cuda", init_values=vals)
batch = data.synthetic_batch(hp, 3, N=17, T=24, shape="ljs", seed=0)
gb = {k: torch.tensor(v).cuda() for k, v in batch.items()}
out, sv = m.forward(gb, None, training=False)
m.backward(sv)
torch.cuda.synchronize()
grads = m.grads_dict()
p64 = {k: v.requires_grad_(True) for k, v in O.to_torch(vals).items()}
ref = O.model_forward(p64, O.to_torch(params.init_bn_buffers(hp)), hp, O.to_torch(batch), None,
                      training=False)
ref["loss"].backward()
gmax = max(float(p.grad.abs().max()) for p in p64.values())
for name, p in p64.items():
    g_ref = p.grad.numpy()
    scale = max(np.abs(g_ref).max(), 1e-4 * gmax)
    err = np.abs(grads[name].astype(np.float64) - g_ref).max() / scale
    if err > 2e-4:
        print(f"{name:60s} {err:.3e}")
print("done", os.environ.get("SAT_MHA_WGRAD_AUX"), os.environ.get("SAT_LIB_OVERRIDE", "in-tree"))
