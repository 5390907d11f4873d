"""Decoder teacher-forced loop on the HIP path vs the CPU oracle (same weights, same masks)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda, B=3, N=23, T=24, seed=0, train=True, lengths=None):
    from sat_amd import hparams, params, data
    from oracle import sat_oracle as O
    hp = hparams.ljspeech_hparams()
    d = params.resolve_dims(hp)
    vals = params.init_params(hp, seed=7)
    L = params.Layout(params.param_specs(hp))
    flat = torch.tensor(L.pack(vals)).to(cuda)
    P = L.views(flat)
    rng = np.random.default_rng(seed)
    lens = np.array(lengths if lengths is not None else rng.integers(N // 2, N + 1, B), np.int64)
    lens[0] = N
    m1 = rng.standard_normal((B, N, d.m1)).astype(np.float32) * 0.5
    m2 = rng.standard_normal((B, N, d.m2)).astype(np.float32) * 0.5
    tgt = rng.standard_normal((B, T, hp.num_mels)).astype(np.float32)
    masks = None
    if train:
        masks = {k: v for k, v in data.synthetic_masks(hp, B, N, T // hp.outputs_per_step,
                                                       seed=seed + 1).items()
                 if k.startswith("dec/") and "sa" not in k}
    return hp, d, vals, P, lens, m1, m2, tgt, masks, O


@pytest.mark.parametrize("train", [False, True])
def test_decoder_loop_matches_oracle(cuda, train):
    from sat_amd import decoder
    hp, d, vals, P, lens, m1, m2, tgt, masks, O = _setup(cuda, train=train)
    dm = None if masks is None else {k: torch.tensor(v).to(cuda) for k, v in masks.items()}
    D, sv = decoder.decoder_forward(P, hp, d, torch.tensor(m1).to(cuda), torch.tensor(m2).to(cuda),
                                    torch.tensor(lens).to(cuda), torch.tensor(tgt).to(cuda), dm)
    torch.cuda.synchronize()
    p64 = O.to_torch(vals)
    om = None if masks is None else O.to_torch(masks)
    ref, extra = O.decoder_loop(torch.tensor(m1).double(), torch.tensor(m2).double(),
                                torch.tensor(lens), torch.tensor(tgt).double(), p64, hp, om,
                                record=True)
    A, M1, M2 = d.att_rnn, d.m1, d.m2
    h0 = sv.H0RAW.transpose(0, 1).double().cpu()
    np.testing.assert_allclose(h0.numpy(), extra["h0"].numpy(), rtol=0, atol=2e-5)
    ctx = sv.REC0[1:, :, :M1].transpose(0, 1).double().cpu()
    np.testing.assert_allclose(ctx.numpy(), extra["c1"].numpy(), rtol=0, atol=2e-5)
    c2 = sv.REC0[1:, :, M1:M1 + M2].transpose(0, 1).double().cpu()
    np.testing.assert_allclose(c2.numpy(), extra["c2"].numpy(), rtol=0, atol=2e-5)
    al = sv.AL1[1:].transpose(0, 1).double().cpu()
    np.testing.assert_allclose(al.numpy(), extra["alignment1"].numpy(), rtol=0, atol=2e-5)
    s2 = sv.S2.transpose(0, 1).double().cpu()
    np.testing.assert_allclose(s2.numpy(), extra["alignment2"].numpy(), rtol=0, atol=2e-5)
    out = D.transpose(0, 1).double().cpu()
    err = (out - ref).abs()
    assert float(err.mean()) < 1e-5 and float(err.max()) < 1e-4
