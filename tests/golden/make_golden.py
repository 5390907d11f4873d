"""Generate the golden fixtures under tests/golden/ from the CPU oracle (float64).

    python tests/golden/make_golden.py

The reference (TF1.x + tacotron2@6af04c7) cannot run in this image and ships no golden vectors
(SURVEY.md section 8(c)), so these vectors are the oracle's: they freeze the restatement's
numbers (a regression pin for the oracle, checked by tests/test_golden_cpu.py) and give the HIP
path fixed inputs/expected outputs (tests/test_golden_gpu.py).  Parity against true TF numbers
stays unpinned, as documented in DESIGN.md.

Files:
  golden_model.npz  -- LJSpeech hparams, weights init_params(seed=5), one ragged batch
                       (B=2, N=12, T=16, r=2), its dropout/zoneout masks, and the oracle's
                       eval- and train-mode outputs + per-parameter gradient summaries.
  golden_model_vctk.npz -- the same for the VCTK multi-speaker config (speaker Embedding
                       152x16 offset 225 -> MultiSpeakerPreNet), B=3, N=10, T=12.
  golden_ops.npz    -- single-op vectors: zoneout LSTM step (train/eval), causal MHA,
                       SAME conv with an even kernel, MaxPool(2,1,SAME), the loss.
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import _sat_path  # noqa: E402

_sat_path.load()
from sat_amd import data, hparams, params  # noqa: E402
from oracle import sat_oracle as O  # noqa: E402

MODEL_CASES = {
    "ljspeech": dict(B=2, N=12, T=16, shape="ljs", batch_seed=1, mask_seed=7, init_seed=5,
                     file="golden_model.npz"),
    "vctk": dict(B=3, N=10, T=12, shape="ljs", batch_seed=4, mask_seed=8, init_seed=5,
                 file="golden_model_vctk.npz"),
}
MODEL_CASE = MODEL_CASES["ljspeech"]
N_HEAD = 8   # leading gradient entries stored per parameter


def model_case(preset="ljspeech"):
    c = MODEL_CASES[preset]
    hp = getattr(hparams, f"{preset}_hparams")()
    vals = params.init_params(hp, seed=c["init_seed"])
    batch = data.synthetic_batch(hp, c["B"], N=c["N"], T=c["T"], shape=c["shape"],
                                 seed=c["batch_seed"])
    Np, Tp = batch["source"].shape[1], batch["mel"].shape[1] // hp.outputs_per_step
    masks = data.synthetic_masks(hp, c["B"], Np, Tp, seed=c["mask_seed"])
    return hp, vals, batch, masks


def param_checksums(vals):
    names = sorted(vals)
    arr = {k: np.asarray(vals[k], np.float64) for k in names}
    return names, np.array([[arr[k].sum(), np.abs(arr[k]).sum()] for k in names])


def oracle_model(hp, vals, batch, masks, training):
    p64 = {k: v.requires_grad_(True) for k, v in O.to_torch(vals).items()}
    bufs = O.to_torch(params.init_bn_buffers(hp))
    ref = O.model_forward(p64, bufs, hp, O.to_torch(batch),
                          O.to_torch(masks) if training else None, training=training)
    ref["loss"].backward()
    names = sorted(p64)
    gsum = np.array([[float(p64[k].grad.sum()), float((p64[k].grad ** 2).sum())] for k in names])
    ghead = np.zeros((len(names), N_HEAD))
    for i, k in enumerate(names):
        g = p64[k].grad.reshape(-1).numpy()
        ghead[i, :min(N_HEAD, g.size)] = g[:N_HEAD]
    return {"loss": float(ref["loss"].detach()), "l1": float(ref["l1"].detach()),
            "bce": float(ref["bce"].detach()), "mel": ref["mel"].detach().numpy(),
            "stop": ref["stop"].detach().numpy(), "grad_sum_sumsq": gsum, "grad_head": ghead}


def ops_case():
    rng = np.random.default_rng(2024)
    f = lambda *s: rng.standard_normal(s)  # noqa: E731
    out = {}
    # zoneout LSTM step: x [3,10], state [3,6], W [16, 24]
    x, c, h = f(3, 10), f(3, 6), f(3, 6)
    w, b = 0.3 * f(16, 24), 0.1 * f(24)
    mc = (rng.random((3, 6)) < 0.9).astype(np.float64)
    mh = (rng.random((3, 6)) < 0.9).astype(np.float64)
    T = lambda a: torch.tensor(a)  # noqa: E731
    for mode, (m1, m2) in {"train": (T(mc), T(mh)), "eval": (None, None)}.items():
        hr, c2, h2 = O.zoneout_lstm_step(T(x), T(c), T(h), T(w), T(b), 0.1, 0.1, m1, m2)
        out[f"zlstm_{mode}_out"] = np.stack([hr.numpy(), c2.numpy(), h2.numpy()])
    out.update(zlstm_x=x, zlstm_c=c, zlstm_h=h, zlstm_w=w, zlstm_b=b, zlstm_mc=mc, zlstm_mh=mh)
    # causal MHA: x [2,5,8], 2 heads
    xm = f(2, 5, 8)
    pm = {}
    for nm in ("query_projection", "key_projection", "value_projection", "output_projection"):
        pm[f"mha/{nm}/kernel"] = 0.4 * f(8, 8)
        pm[f"mha/{nm}/bias"] = 0.1 * f(8)
    y, a = O.mha(T(xm), {k: T(v) for k, v in pm.items()}, "mha", 2, True, None)
    out.update(mha_x=xm, mha_out=y.numpy(), mha_probs=a.numpy(),
               **{f"mha_p_{k.replace('/', '__')}": v for k, v in pm.items()})
    # SAME conv, even kernel (pad_left = 4, pad_right = 5), and MaxPool(2,1,SAME)
    xc, wc, bc = f(2, 7, 3), f(10, 3, 4), f(4)
    out.update(conv_x=xc, conv_w=wc, conv_b=bc,
               conv_out=O.conv1d_same(T(xc), T(wc), T(bc)).numpy(),
               pool_out=O.maxpool2_same(T(xc)).numpy())
    # loss: 0.1 * L1 + BCE, SUM_BY_NONZERO_WEIGHTS
    mel, tgt = f(2, 6, 4), f(2, 6, 4)
    stop = f(2, 3, 1)
    tmask = np.array([[1, 1, 1, 1, 0, 0], [1, 1, 1, 1, 1, 1]], np.float64)
    done = np.array([[0, 1, 1], [0, 0, 1]], np.float64)
    dmask = np.array([[1, 1, 0], [1, 1, 1]], np.float64)
    loss, l1, bce = O.losses(T(mel), T(stop), T(tgt), T(tmask), T(done), T(dmask))
    out.update(loss_mel=mel, loss_stop=stop, loss_tgt=tgt, loss_tmask=tmask, loss_done=done,
               loss_dmask=dmask, loss_out=np.array([float(loss), float(l1), float(bce)]))
    return out


def main():
    for preset, c in MODEL_CASES.items():
        hp, vals, batch, masks = model_case(preset)
        names, cks = param_checksums(vals)
        rec = {"param_names": np.array(names), "param_checksums": cks}
        rec.update({f"batch__{k}": v for k, v in batch.items()})
        rec.update({f"mask__{k}": v for k, v in masks.items()})
        for mode in ("eval", "train"):
            r = oracle_model(hp, vals, batch, masks, mode == "train")
            for k, v in r.items():
                rec[f"{mode}__{k}"] = np.asarray(v)
        np.savez_compressed(os.path.join(HERE, c["file"]), **rec)
        print("wrote", c["file"])
    np.savez_compressed(os.path.join(HERE, "golden_ops.npz"), **ops_case())
    print("wrote golden_ops.npz")


if __name__ == "__main__":
    main()
