"""CPU tests of the oracle restatement (no GPU).

The reference's only behavioural test, ``modules/transformer_test.py:44-90``, asserts that the
RNNTransformer training branch (loop, then post-hoc causal self-attention) equals the
teacher-forced incremental branch (self-attention re-run over the growing history) -- ported
here as a hypothesis property on the oracle, plus unit checks of the TF semantics the oracle
restates.
"""
import numpy as np
import pytest
import torch
from hypothesis import given, settings, strategies as st

from oracle import sat_oracle as O


def _sa_params(dim, heads, seed):
    g = torch.Generator().manual_seed(seed)
    p = {}
    for name in ("query", "key", "value", "output"):
        p[f"decoder/self_attention0/mha/{name}_projection/kernel"] = \
            torch.randn(dim, dim, generator=g, dtype=torch.float64) / dim ** 0.5
        p[f"decoder/self_attention0/mha/{name}_projection/bias"] = \
            torch.randn(dim, generator=g, dtype=torch.float64) * 0.1
    p["decoder/self_attention0/transform/kernel"] = torch.randn(dim, dim, generator=g,
                                                                dtype=torch.float64) / dim ** 0.5
    p["decoder/self_attention0/transform/bias"] = torch.zeros(dim, dtype=torch.float64)
    return p


@settings(max_examples=25, deadline=None)
@given(batch=st.integers(1, 3), dim=st.integers(1, 10).map(lambda x: 2 * x),
       t_factor=st.integers(2, 8), r=st.integers(1, 2), seed=st.integers(0, 2 ** 16))
def test_equality_between_training_and_inference(batch, dim, t_factor, r, seed):
    """modules/transformer_test.py:44-90: one-hot targets, plain LSTMCell(dim*r) decoder cell,
    RNNTransformer with 2 heads and dropout 0; training branch == incremental branch."""
    from sat_amd import hparams
    rng = np.random.default_rng(seed)
    T = t_factor * r
    ids = rng.integers(0, dim, size=(batch, T))
    tgt = torch.zeros(batch, T, dim, dtype=torch.float64)
    tgt.scatter_(2, torch.tensor(ids).unsqueeze(-1), 1.0)
    units = dim * r
    hp = hparams.ljspeech_hparams(num_mels=dim, outputs_per_step=r, n_feed_frame=r,
                                  decoder_self_attention_num_heads=2,
                                  decoder_self_attention_out_units=units, decoder_out_units=units)
    p = _sa_params(units, 2, seed)
    g = torch.Generator().manual_seed(seed + 1)
    p["decoder/out_projection/kernel"] = torch.randn(units, dim * r, generator=g, dtype=torch.float64)
    p["decoder/out_projection/bias"] = torch.zeros(dim * r, dtype=torch.float64)
    p["decoder/stop_token_projection/kernel"] = torch.randn(units, 1, generator=g, dtype=torch.float64)
    p["decoder/stop_token_projection/bias"] = torch.zeros(1, dtype=torch.float64)
    W = torch.randn(dim * r + units, 4 * units, generator=g, dtype=torch.float64) * 0.3
    bvec = torch.zeros(4 * units, dtype=torch.float64)
    x = O.teacher_inputs(tgt, r, r)
    c = h = torch.zeros(batch, units, dtype=torch.float64)
    outs = []
    for t in range(x.shape[1]):
        h, c = O.lstm_cell(x[:, t], c, h, W, bvec)
        outs.append(h)
    dout = torch.stack(outs, 1)
    mel_t, stop_t, _ = O.decoder_head(dout, p, hp, None)
    mel_i, stop_i = O.decoder_head_incremental(dout, p, hp)
    np.testing.assert_allclose(mel_t.numpy(), mel_i.numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(stop_t.numpy(), stop_i.numpy(), rtol=1e-6, atol=1e-6)
    # argmax samples (modules/module.py:760-763)
    s_t = mel_t.view(batch, -1, r, dim).argmax(-1)
    s_i = mel_i.view(batch, -1, r, dim).argmax(-1)
    assert torch.equal(s_t, s_i)


def test_full_model_training_equals_incremental_head():
    from sat_amd import hparams, params, data
    hp = hparams.ljspeech_hparams()
    p = O.to_torch(params.init_params(hp, seed=3))
    bufs = O.to_torch(params.init_bn_buffers(hp))
    b = O.to_torch(data.synthetic_batch(hp, 2, N=9, T=12, shape="ljs", seed=1))
    out = O.model_forward(p, bufs, hp, b, None, training=False)
    mel_i, stop_i = O.decoder_head_incremental(out["dout"], p, hp)
    np.testing.assert_allclose(out["mel"].reshape(mel_i.shape).numpy(), mel_i.numpy(),
                               rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(out["stop"].numpy(), stop_i.numpy(), rtol=1e-9, atol=1e-9)


def test_conv1d_same_padding_even_kernel():
    # TF SAME for k=10: pad_left = 4, pad_right = 5 (cross-correlation)
    x = torch.zeros(1, 12, 1, dtype=torch.float64)
    x[0, 6, 0] = 1.0
    w = torch.arange(10, dtype=torch.float64).view(10, 1, 1)
    y = O.conv1d_same(x, w, None)[0, :, 0]
    # y[n] = sum_j x[n + j - 4] w[j]  ->  nonzero where n + j - 4 == 6  ->  y[n] = w[10 - n]
    expect = torch.tensor([0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0], dtype=torch.float64)
    for n in range(12):
        j = 6 + 4 - n
        if 0 <= j < 10:
            expect[n] = j
    assert torch.equal(y, expect)


def test_maxpool_same():
    x = torch.tensor([[[1.0], [3.0], [2.0], [0.0]]], dtype=torch.float64)
    assert O.maxpool2_same(x)[0, :, 0].tolist() == [3.0, 3.0, 2.0, 0.0]


def test_zoneout_eval_blend_and_masks():
    g = torch.Generator().manual_seed(0)
    x, c, h = (torch.randn(2, 3, generator=g, dtype=torch.float64) for _ in range(3))
    W = torch.randn(6, 12, generator=g, dtype=torch.float64)
    b = torch.zeros(12, dtype=torch.float64)
    hr, cr = O.lstm_cell(x, c, h, W, b)
    out, c2, h2 = O.zoneout_lstm_step(x, c, h, W, b, 0.1, 0.1, None, None)
    assert torch.allclose(out, hr)
    assert torch.allclose(c2, 0.9 * cr + 0.1 * c) and torch.allclose(h2, 0.9 * hr + 0.1 * h)
    m = torch.tensor([[1.0, 0.0, 1.0], [0.0, 1.0, 0.0]], dtype=torch.float64)
    _, c3, h3 = O.zoneout_lstm_step(x, c, h, W, b, 0.1, 0.1, m, m)
    assert torch.allclose(c3, m * cr + (1 - m) * c) and torch.allclose(h3, m * hr + (1 - m) * h)


def test_forward_attention_properties():
    """alpha sums to 1, is exactly 0 past the memory length, and starts monotonic at n=0."""
    from sat_amd import hparams, params
    hp = hparams.ljspeech_hparams()
    p = O.to_torch(params.init_params(hp, seed=1))
    g = torch.Generator().manual_seed(0)
    mem = torch.randn(2, 11, 256, generator=g, dtype=torch.float64)
    lens = torch.tensor([11, 6])
    att = O.ForwardAttentionOracle(p, "decoder/attention1", mem, lens)
    st_ = att.initial_state(2, 11, torch.float64)
    for _ in range(5):
        q = torch.randn(2, 256, generator=g, dtype=torch.float64)
        a, st_ = att(q, st_)
        assert torch.allclose(a.sum(1), torch.ones(2, dtype=torch.float64))
        assert float(a[1, 6:].abs().max()) == 0.0
    # after one step from alpha_0 = onehot(0), mass can only be at n in {0, 1} up to the 1e-7 floor
    st0 = att.initial_state(2, 11, torch.float64)
    a1, _ = att(torch.zeros(2, 256, dtype=torch.float64), st0)
    assert float(a1[:, 2:].sum()) < 1e-4


def test_losses_sum_by_nonzero_weights():
    mel = torch.zeros(1, 4, 2, dtype=torch.float64)
    tgt = torch.ones(1, 4, 2, dtype=torch.float64)
    mask = torch.tensor([[1.0, 1.0, 0.0, 0.0]], dtype=torch.float64)
    stop = torch.zeros(1, 2, 1, dtype=torch.float64)
    done = torch.tensor([[0.0, 1.0]], dtype=torch.float64)
    dmask = torch.tensor([[1.0, 0.0]], dtype=torch.float64)
    loss, l1, bce = O.losses(mel, stop, tgt, mask, done, dmask)
    assert float(l1) == pytest.approx(1.0)
    assert float(bce) == pytest.approx(np.log(2.0))
    assert float(loss) == pytest.approx(0.1 + np.log(2.0))


def test_learning_rate_and_adam():
    assert O.learning_rate(5e-4, 0) == pytest.approx(5e-4 * 4000 ** 0.5 * 4000 ** -1.5)
    assert O.learning_rate(5e-4, 3999) == pytest.approx(5e-4 * 4000 ** 0.5 * 4000 ** -0.5)
    assert O.learning_rate(5e-4, 15999) < O.learning_rate(5e-4, 3999)
    p = torch.ones(3, dtype=torch.float64)
    g = torch.tensor([1.0, -2.0, 0.0], dtype=torch.float64)
    p2, m, v = O.adam_tf(p, g, torch.zeros(3, dtype=torch.float64),
                         torch.zeros(3, dtype=torch.float64), 0.1, 1)
    # first step of TF Adam moves every non-zero-gradient coordinate by ~lr against the sign
    assert torch.allclose(p2[:2], torch.tensor([0.9, 1.1], dtype=torch.float64), atol=1e-6)
    clipped, norm = O.clip_by_global_norm([torch.tensor([3.0, 4.0])], 1.0)
    assert norm == pytest.approx(5.0) and torch.allclose(clipped[0], torch.tensor([0.6, 0.8]))


def test_oracle_gradients_flow_everywhere():
    from sat_amd import hparams, params, data
    hp = hparams.ljspeech_hparams()
    p = {k: v.requires_grad_(True) for k, v in O.to_torch(params.init_params(hp)).items()}
    bufs = O.to_torch(params.init_bn_buffers(hp))
    b = O.to_torch(data.synthetic_batch(hp, 2, N=8, T=8, shape="max", seed=2))
    m = O.to_torch(data.synthetic_masks(hp, 2, 8, 4, seed=3))
    out = O.model_forward(p, bufs, hp, b, m, training=True)
    out["loss"].backward()
    missing = [k for k, v in p.items() if v.grad is None]
    assert missing == []


def test_oracle_kinks_from_its_own_forward_change_nothing():
    """encoder(kinks=) with the gates / pool choices the float64 forward itself takes gives the
    kink-free forward and gradients bit for bit (the option only fixes WHICH branch is taken at
    a ReLU / max-pool kink; tests/test_fullshape_gpu.py feeds it the HIP forward's branches)."""
    from sat_amd import hparams, params, data
    hp = hparams.ljspeech_hparams()
    vals = params.init_params(hp, seed=5)
    bufs = O.to_torch(params.init_bn_buffers(hp))
    b = O.to_torch(data.synthetic_batch(hp, 2, N=9, T=8, shape="ljs", seed=2))
    m = O.to_torch(data.synthetic_masks(hp, 2, b["source"].shape[1], 4, seed=3))
    # the float64 forward's own branches (the helper the C2 gradient test bounds flips with)
    kinks = O.encoder_front_branches(b["source"], O.to_torch(vals), bufs, hp, m, True)
    res = []
    for kk in (None, kinks):
        p = {k: v.clone().requires_grad_(True) for k, v in O.to_torch(vals).items()}
        out = O.model_forward(p, bufs, hp, b, m, training=True, kinks=kk)
        out["loss"].backward()
        res.append((out["mel"].detach(), {k: v.grad for k, v in p.items()}))
    (mel_a, g_a), (mel_b, g_b) = res
    assert torch.equal(mel_a, mel_b)
    for k in g_a:
        assert torch.allclose(g_a[k], g_b[k], rtol=0, atol=1e-12 * float(g_a[k].abs().max()) + 1e-300), k


@pytest.mark.parametrize("preset", ["ljspeech", "vctk"])
def test_free_running_equals_teacher_forced_on_its_own_predictions(preset):
    """The PREDICT restatement (StopTokenBasedInferenceHelper feeding back the last predicted
    frame + TransformerWrapper re-running the causal self-attention over the history) equals
    the teacher-forced eval path (TransformerTrainingHelper + post-hoc causal self-attention,
    modules/module.py:743-764) when the teacher frames ARE the free-running predictions --
    exactly the modules/transformer_test.py:44-90 equivalence, closed over the feedback loop."""
    from sat_amd import data, hparams, params
    hp = getattr(hparams, f"{preset}_hparams")()
    vals = params.init_params(hp, seed=5)
    p = O.to_torch(vals)
    bufs = O.to_torch(params.init_bn_buffers(hp))
    b = O.to_torch(data.synthetic_batch(hp, 2, N=9, T=16, shape="ljs", seed=3))
    inf = O.infer_free_running(p, bufs, hp, b, max_iters=8, min_iters=100)
    assert inf["steps"] == 8
    tb = dict(b)
    T = inf["mel"].shape[1]
    tb["mel"] = inf["mel"]
    tb["mel_mask"] = torch.ones(2, T, dtype=torch.float64)
    tb["done"] = torch.zeros(2, T // hp.outputs_per_step, dtype=torch.float64)
    tb["done_mask"] = torch.ones_like(tb["done"])
    tf = O.model_forward(p, bufs, hp, tb, None, training=False)
    np.testing.assert_allclose(tf["mel"].numpy(), inf["mel"].numpy(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(tf["stop"][..., 0].numpy(), inf["stop"].numpy(), rtol=1e-10,
                               atol=1e-12)
    np.testing.assert_allclose(tf["alignment1"].numpy(), inf["alignment1"].numpy(), atol=1e-12)


def test_free_running_stop_rule():
    """is_finished: t > min_iters and sigmoid(stop) > 0.5 for every utterance (reduce_all)."""
    from sat_amd import data, hparams, params
    hp = hparams.ljspeech_hparams()
    vals = params.init_params(hp, seed=5)
    bufs = O.to_torch(params.init_bn_buffers(hp))
    b = O.to_torch(data.synthetic_batch(hp, 2, N=7, T=8, shape="ljs", seed=1))
    for bias, steps in ((9.0, 6), (-9.0, 15)):
        vals["decoder/stop_token_projection/bias"] = np.full((1,), bias, np.float32)
        out = O.infer_free_running(O.to_torch(vals), bufs, hp, b, max_iters=15, min_iters=4)
        assert out["steps"] == steps


def test_forced_alignment_replay_equals_free_running():
    """Forced-alignment pass (TeacherForcing*Attention, modules/teacher_forcing_attention.py:
    30-35) replaying the alignments a free-running decode computed, with the same feedback,
    reproduces that decode: the teacher mechanisms return exactly what the real ones did."""
    from sat_amd import data, hparams, params
    hp = hparams.ljspeech_hparams()
    p = O.to_torch(params.init_params(hp, seed=5))
    bufs = O.to_torch(params.init_bn_buffers(hp))
    b = O.to_torch(data.synthetic_batch(hp, 2, N=9, T=16, shape="ljs", seed=3))
    inf = O.infer_free_running(p, bufs, hp, b, max_iters=8, min_iters=100)
    fa = O.infer_free_running(p, bufs, hp, b, forced=(inf["alignment1"], inf["alignment2"]))
    assert fa["steps"] == 8
    np.testing.assert_allclose(fa["mel"].numpy(), inf["mel"].numpy(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(fa["stop"].numpy(), inf["stop"].numpy(), rtol=1e-12, atol=1e-12)


def test_forced_alignment_softmax_feedback():
    """OneHotValidationHelper(teacher_forcing=False) (modules/helpers.py:96-108): step t+1 is fed
    softmax over the bins of step t's last frame, T' steps exactly, stop tokens ignored."""
    from sat_amd import data, hparams, params
    hp = hparams.ljspeech_hparams()
    vals = params.init_params(hp, seed=5)
    vals["decoder/stop_token_projection/bias"] = np.full((1,), 9.0, np.float32)  # would stop
    p = O.to_torch(vals)
    bufs = O.to_torch(params.init_bn_buffers(hp))
    b = O.to_torch(data.synthetic_batch(hp, 2, N=9, T=16, shape="ljs", seed=3))
    tf = O.model_forward(p, bufs, hp, b, None, training=False)
    a1, a2 = tf["alignment1"], tf["alignment2"]
    fa = O.infer_free_running(p, bufs, hp, b, forced=(a1, a2), feed="softmax", min_iters=0)
    assert fa["steps"] == a1.shape[1] == 8
    M, r = hp.num_mels, hp.outputs_per_step
    # step 0 sees the go frame and the teacher-forced alpha_0: identical to the teacher-forced
    # pass; from step 1 the fed frames differ (softmax vs target)
    np.testing.assert_allclose(fa["mel"][:, :r].numpy(), tf["mel"][:, :r].numpy(), atol=1e-12)
    assert not np.allclose(fa["mel"][:, r:2 * r].numpy(), tf["mel"][:, r:2 * r].numpy())
    assert torch.isfinite(fa["mel"]).all() and fa["mel"].shape == (2, 16, M)
