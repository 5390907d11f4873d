"""Full teacher-forced forward (encoder + decoder + heads + loss) on HIP vs the CPU oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def build(cuda, hp, B, N, T, seed=0, train=False, shape="ljs"):
    from sat_amd import params, data, kernels, model
    from oracle import sat_oracle as O
    d = params.resolve_dims(hp)
    vals = params.init_params(hp, seed=11)
    L = params.Layout(params.param_specs(hp))
    flat = torch.tensor(L.pack(vals)).to(cuda)
    P = L.views(flat)
    bn = model.BNState(hp, cuda)
    batch = data.synthetic_batch(hp, B, N=N, T=T, shape=shape, seed=seed)
    masks = data.synthetic_masks(hp, B, batch["source"].shape[1],
                                 batch["mel"].shape[1] // hp.outputs_per_step,
                                 seed=seed + 5) if train else None
    return d, vals, P, bn, batch, masks, O


@pytest.mark.parametrize("train", [False, True])
def test_model_forward_matches_oracle(cuda, train):
    from sat_amd import hparams, kernels, model
    hp = hparams.ljspeech_hparams()
    d, vals, P, bn, batch, masks, O = build(cuda, hp, B=3, N=21, T=30, train=train)
    gb = {k: torch.tensor(v).to(cuda) for k, v in batch.items()}
    gm = None if masks is None else {k: torch.tensor(v).to(cuda) for k, v in masks.items()}
    ws = kernels.Workspace(cuda)
    out, sv = model.model_forward(P, bn, hp, d, gb, gm, training=train, ws=ws)
    torch.cuda.synchronize()
    assert int(sv["emb_err"].item()) == 0
    p64 = O.to_torch(vals)
    from sat_amd import params
    bufs = O.to_torch(params.init_bn_buffers(hp))
    ref = O.model_forward(p64, bufs, hp, O.to_torch(batch),
                          None if masks is None else O.to_torch(masks), training=train)
    m1 = out["m1"].double().cpu()
    assert float((m1 - ref["m1"]).abs().max()) < 5e-5
    m2 = out["m2"].double().cpu()
    assert float((m2 - ref["m2"]).abs().max()) < 5e-5
    mel = out["mel"].double().cpu()
    err = (mel - ref["mel"]).abs()
    assert float(err.mean()) < 1e-5, float(err.mean())
    assert float(err.max()) < 2e-4
    stop = out["stop"].double().cpu()
    assert float((stop - ref["stop"]).abs().max()) < 2e-4
    assert abs(float(out["loss"].item()) - float(ref["loss"])) < 1e-5
    if train:  # BN moving statistics were updated
        assert float(bn.mean.abs().sum()) > 0
