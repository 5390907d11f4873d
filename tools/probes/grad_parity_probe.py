"""Per-parameter gradient error of the HIP training step vs float64 autograd for a few
(B, shape, seed) cases -- locates which rows of the BPTT drift at the benched batch size.

Usage: python tools/probes/grad_parity_probe.py [B:shape:seed ...]   (default 32:max:51 8:max:51 32:ljs:51)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _sat_path  # noqa: E402

_sat_path.load()
from test_fullshape_gpu import _run  # noqa: E402

cases = sys.argv[1:] or ["32:max:51", "8:max:51", "32:ljs:51"]
cuda = torch.device("cuda:0")
for c in cases:
    B, shape, seed = c.split(":")
    hp, m, out, ref, p64, b = _run(cuda, int(B), 200, 1000, True, shape=shape, seed=int(seed),
                                   grads=True)
    grads = m.grads_dict()
    gmax = max(float(p.grad.abs().max()) for p in p64.values())
    rows = []
    for name, p in p64.items():
        g_ref = p.grad.numpy()
        scale = max(np.abs(g_ref).max(), 1e-4 * gmax)
        d = np.abs(grads[name].astype(np.float64) - g_ref)
        fro = float(np.sqrt((d ** 2).sum()) / max(np.sqrt((g_ref ** 2).sum()), 1e-30))
        rows.append((float(d.max() / scale), name, float(np.abs(g_ref).max()), float(d.mean() / scale),
                     fro))
    rows.sort(reverse=True)
    mel = out["mel"].double().cpu().numpy()
    print(f"== B={B} shape={shape} seed={seed}: loss {float(out['loss']):.9g} ref "
          f"{float(ref['loss']):.9g}, mel max {np.abs(mel - ref['mel'].detach().numpy()).max():.3e}, "
          f"gmax {gmax:.3e}", flush=True)
    for r in rows[:40]:
        print(f"  {r[0]:.3e} (mean {r[3]:.2e}, rel-Frobenius {r[4]:.2e}, |g|max {r[2]:.3e})  {r[1]}",
              flush=True)
    del m, out, ref, p64
    torch.cuda.empty_cache()
