"""HIP path (through libsat_hip.so) on the committed golden inputs vs the committed golden
outputs (tests/golden/golden_model.npz): loss, mel, stop tokens and every parameter gradient's
sum / sum-of-squares / leading entries, eval and train (fixed dropout + zoneout masks)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FILES = {"ljspeech": "golden_model.npz", "vctk": "golden_model_vctk.npz"}


@pytest.mark.parametrize("preset", sorted(FILES))
@pytest.mark.parametrize("mode", ["eval", "train"])
def test_hip_path_matches_golden(cuda, mode, preset):
    from sat_amd import engine, hparams, params
    G = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                             FILES[preset]))
    hp = getattr(hparams, f"{preset}_hparams")()
    vals = params.init_params(hp, seed=5)
    names = sorted(vals)
    assert list(G["param_names"]) == names
    np.testing.assert_allclose([np.asarray(vals[k], np.float64).sum() for k in names],
                               G["param_checksums"][:, 0], rtol=1e-12, atol=1e-9)
    batch = {k[len("batch__"):]: G[k] for k in G.files if k.startswith("batch__")}
    masks = {k[len("mask__"):]: G[k].astype(np.float32) for k in G.files
             if k.startswith("mask__")}
    m = engine.Tacotron(hp, cuda, init_values=vals)
    gb = {k: torch.tensor(v).to(cuda) for k, v in batch.items()}
    gm = {k: torch.tensor(v).to(cuda) for k, v in masks.items()} if mode == "train" else None
    out, sv = m.forward(gb, gm, training=mode == "train")
    m.backward(sv)
    torch.cuda.synchronize()
    # fp32 vs float64 oracle tolerances
    assert abs(float(out["loss"].item()) - float(G[f"{mode}__loss"])) < 1e-5
    np.testing.assert_allclose(out["mel"].cpu().numpy(), G[f"{mode}__mel"], atol=2e-5)
    np.testing.assert_allclose(out["stop"].cpu().numpy().reshape(G[f"{mode}__stop"].shape),
                               G[f"{mode}__stop"], atol=2e-5)
    grads = m.grads_dict()
    ref_ss = G[f"{mode}__grad_sum_sumsq"]
    ref_head = G[f"{mode}__grad_head"]
    gmax = float(np.sqrt(ref_ss[:, 1].max()))
    bad = []
    for i, k in enumerate(names):
        g = grads[k].astype(np.float64).reshape(-1)
        n = min(ref_head.shape[1], g.size)
        scale = max(np.sqrt(ref_ss[i, 1]), 1e-4 * gmax)
        e_norm = abs(np.sqrt((g ** 2).sum()) - np.sqrt(ref_ss[i, 1])) / scale
        e_sum = abs(g.sum() - ref_ss[i, 0]) / (scale * np.sqrt(g.size))
        e_head = np.abs(g[:n] - ref_head[i, :n]).max() / scale
        if max(e_norm, e_sum, e_head) > 2e-4:
            bad.append((k, e_norm, e_sum, e_head))
    assert not bad, bad
