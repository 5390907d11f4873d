"""Persistent decoder kernels (sat_decoder_attention_fwd/bwd: all T' steps of attention RNN
+ query + dual-source attention in ONE launch, K/V resident in LDS; sat_decoder_lstms_fwd/bwd:
both decoder LSTM layers in ONE launch; in-kernel group barriers) vs the per-step launch path
and vs the CPU oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(cuda, B, N, T, train, seed=3):
    from sat_amd import data, engine, hparams, params
    hp = hparams.ljspeech_hparams()
    vals = params.init_params(hp, seed=5)
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="ljs", seed=seed)
    Np, Tp = b["source"].shape[1], b["mel"].shape[1] // hp.outputs_per_step
    mk = data.synthetic_masks(hp, B, Np, Tp, seed=seed + 1) if train else None
    gb = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
    gm = None if mk is None else {k: torch.tensor(v).to(cuda) for k, v in mk.items()}
    outs = []
    for persistent in (False, True):
        m = engine.Tacotron(hp, cuda, init_values=vals, persistent_decoder=persistent)
        out, sv = m.forward(gb, gm, training=train)
        m.backward(sv)
        torch.cuda.synchronize()
        if persistent:
            sv["dec"].tensors["attn_scratch"].check()
        outs.append((m, out, sv))
    return hp, vals, b, mk, outs


@pytest.mark.parametrize("B,N,T,train", [(8, 40, 24, True), (32, 200, 60, True),
                                         (16, 71, 30, False), (24, 9, 16, True)])
def test_persistent_equals_per_step(cuda, B, N, T, train):
    hp, vals, b, mk, outs = _pair(cuda, B, N, T, train)
    (m0, o0, s0), (m1, o1, s1) = outs
    assert "attn_scratch" in s1["dec"].tensors and "attn_scratch" not in s0["dec"].tensors
    np.testing.assert_allclose(o1["mel"].cpu().numpy(), o0["mel"].cpu().numpy(), atol=2e-5)
    np.testing.assert_allclose(o1["stop"].cpu().numpy(), o0["stop"].cpu().numpy(), atol=2e-5)
    assert abs(float(o1["loss"].item()) - float(o0["loss"].item())) < 1e-5
    for name in ("REC0", "C0", "H0RAW", "G0", "Q", "S1", "AL1", "S2", "LOC",
                 "H1RAW", "C1S", "H1S", "G1", "H2RAW", "C2S", "H2S", "G2"):
        a, r = s1["dec"].tensors[name], s0["dec"].tensors[name]
        np.testing.assert_allclose(a.cpu().numpy(), r.cpu().numpy(), atol=2e-5, err_msg=name)
    st0, st1 = s0["dec"].tensors["ST"], s1["dec"].tensors["ST"]
    np.testing.assert_allclose(st1[..., 2].cpu().numpy(), st0[..., 2].cpu().numpy(), rtol=1e-5)
    g0, g1 = m0.grads.cpu().numpy(), m1.grads.cpu().numpy()
    assert np.abs(g1 - g0).max() <= 1e-4 * np.abs(g0).max()


def test_persistent_gradients_match_oracle(cuda):
    from sat_amd import params
    from oracle import sat_oracle as O
    hp, vals, b, mk, outs = _pair(cuda, 8, 17, 16, True, seed=7)
    m, out, sv = outs[1]
    grads = m.grads_dict()
    p64 = {k: v.requires_grad_(True) for k, v in O.to_torch(vals).items()}
    ref = O.model_forward(p64, O.to_torch(params.init_bn_buffers(hp)), hp, O.to_torch(b),
                          O.to_torch(mk), training=True)
    ref["loss"].backward()
    assert abs(float(out["loss"].item()) - float(ref["loss"].detach())) < 1e-5
    gmax = max(float(p.grad.abs().max()) for p in p64.values())
    bad = []
    for name, p in p64.items():
        g_ref = p.grad.numpy()
        scale = max(np.abs(g_ref).max(), 1e-4 * gmax)
        err = np.abs(grads[name].astype(np.float64) - g_ref).max() / scale
        if not err < 2e-4:
            bad.append((name, float(err)))
    assert not bad, bad


def test_xcd_store_policy_is_bitwise_neutral(cuda, monkeypatch):
    """The hand-off store policy (persistent.h xcd_local_group: plain stores when the group
    is on one XCD, sc1 otherwise; SAT_XCD_LOCAL=0 forces sc1) changes where lines live, never
    the values: forward outputs and every parameter gradient are bit-identical."""
    from sat_amd import data, engine, hparams, params
    hp = hparams.ljspeech_hparams()
    vals = params.init_params(hp, seed=5)
    b = data.synthetic_batch(hp, 16, N=60, T=40, shape="ljs", seed=9)
    Np, Tp = b["source"].shape[1], b["mel"].shape[1] // hp.outputs_per_step
    mk = data.synthetic_masks(hp, 16, Np, Tp, seed=10)
    gb = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
    gm = {k: torch.tensor(v).to(cuda) for k, v in mk.items()}
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SAT_XCD_LOCAL", flag)
        m = engine.Tacotron(hp, cuda, init_values=vals, persistent_decoder=True)
        out, sv = m.forward(gb, gm, training=True)
        m.backward(sv)
        torch.cuda.synchronize()
        sv["dec"].tensors["attn_scratch"].check()
        res.append((out["mel"].cpu().numpy(), m.grads_dict()))
    (mel_a, g_a), (mel_b, g_b) = res
    np.testing.assert_array_equal(mel_a, mel_b)
    for k in g_a:                   # embedding included: its scatter-add is ordered
        np.testing.assert_array_equal(g_a[k], g_b[k], err_msg=k)
