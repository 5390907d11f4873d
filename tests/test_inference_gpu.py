"""C5 free-running inference (BASELINE configs[4]) on libsat_hip vs the CPU oracle's restatement
of the PREDICT path (oracle.infer_free_running: StopTokenBasedInferenceHelper + TransformerWrapper
re-running the causal self-attention over the whole history; modules/module.py:766-784,
modules/rnn_wrappers.py:87-124, 188-214, helpers analog modules/helpers.py:111-160).

Tolerances: the decode feeds its own predictions back for up to max_iters steps, so fp32 vs
float64 drift compounds through the recurrence; mel frames within 2e-4 absolute over 40 steps."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda, preset="ljspeech", B=3, N=15, seed=2, scale_stop=None):
    from sat_amd import data, engine, hparams, params
    from oracle import sat_oracle as O
    hp = getattr(hparams, f"{preset}_hparams")()
    vals = params.init_params(hp, seed=5)
    if scale_stop is not None:           # bias the stop token so the helper terminates early
        vals["decoder/stop_token_projection/bias"] = np.full((1,), scale_stop, np.float32)
    m = engine.Tacotron(hp, cuda, init_values=vals)
    b = data.synthetic_batch(hp, B, N=N, T=20, shape="ljs", seed=seed)
    gb = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
    p64 = O.to_torch(vals)
    bufs = O.to_torch(params.init_bn_buffers(hp))
    return hp, m, b, gb, p64, bufs, O


@pytest.mark.parametrize("preset", ["ljspeech", "vctk"])
def test_free_running_matches_oracle(cuda, preset):
    from sat_amd.inference import FreeRunningDecoder
    hp, m, b, gb, p64, bufs, O = _setup(cuda, preset)
    T = 40
    out = FreeRunningDecoder(m, max_iters=T, check_every=7).run(gb)
    ref = O.infer_free_running(p64, bufs, hp, O.to_torch(b), max_iters=T)
    assert out["steps"] == ref["steps"]
    np.testing.assert_allclose(out["mel"].cpu().numpy(), ref["mel"].numpy(), atol=2e-4)
    np.testing.assert_allclose(out["stop"].cpu().numpy(), ref["stop"].numpy(), atol=2e-4)
    np.testing.assert_allclose(out["alignment1"].cpu().numpy(),
                               ref["alignment1"].permute(0, 2, 1).numpy(), atol=2e-5)
    np.testing.assert_allclose(out["alignment2"].cpu().numpy(),
                               ref["alignment2"].permute(0, 2, 1).numpy(), atol=2e-5)
    # KV-cached rows == the last step's full causal re-run (TransformerWrapper)
    np.testing.assert_allclose(out["decoder_self_alignments"][0].cpu().numpy(),
                               ref["decoder_self_alignments"][0].numpy(), atol=2e-5)


@pytest.mark.parametrize("bias", [8.0, -8.0])
def test_stop_token_termination(cuda, bias):
    """sigmoid(stop) > 0.5 for all utterances stops the decode right after step min_iters + 1
    (t > min_iters); never > 0.5 runs to max_iters -- the same step count as the oracle."""
    from sat_amd.inference import FreeRunningDecoder
    hp, m, b, gb, p64, bufs, O = _setup(cuda, B=2, N=9, scale_stop=bias)
    out = FreeRunningDecoder(m, max_iters=30, min_iters=10, check_every=4).run(gb)
    ref = O.infer_free_running(p64, bufs, hp, O.to_torch(b), max_iters=30, min_iters=10)
    assert out["steps"] == ref["steps"] == (12 if bias > 0 else 30)
    assert out["mel"].shape[1] == out["steps"] * hp.outputs_per_step
    np.testing.assert_allclose(out["mel"].cpu().numpy(), ref["mel"].numpy(), atol=2e-4)


def test_teacher_forcing_mechanism_replays_alignments(cuda):
    """TeacherForcing*Attention (modules/teacher_forcing_attention.py:30-41): state (alignments,
    index) starts at index -1; call k returns teacher_alignments[:, k], whatever the query."""
    from sat_amd import attentions as A
    from sat_amd import hparams
    hp = hparams.ljspeech_hparams()
    fn1, fn2 = A.force_alignment_dual_source_attention_factory(hp)
    g = torch.Generator().manual_seed(0)
    mem = torch.randn(2, 7, 32, generator=g).to(cuda)
    lens = torch.tensor([7, 4], dtype=torch.int64, device=cuda)
    ta = torch.softmax(torch.randn(2, 5, 7, generator=g), -1).to(cuda)
    mech = fn2(mem, lens, ta)
    assert mech.alignments_size == 7
    np.testing.assert_array_equal(mech.values[1, 4:].cpu().numpy(), 0.0)   # masked memory
    state = mech.initial_state(2)
    assert state[1] == -1
    for k in range(5):
        al, state = mech(torch.randn(2, 256, device=cuda), state)
        assert state[1] == k
        assert torch.equal(al, ta[:, k])
    with pytest.raises(ValueError, match="teacher_alignments"):
        fn1(mem, lens, None)


@pytest.mark.parametrize("preset", ["ljspeech", "vctk"])
def test_forced_alignment_pass_matches_oracle(cuda, preset):
    """use_forced_alignment_mode second pass (models/models.py:118-148): forced alignments from
    the teacher-forced pass, softmax feedback, exactly T' steps; HIP vs the oracle's
    restatement (infer_free_running(forced=..., feed='softmax'))."""
    from sat_amd.inference import FreeRunningDecoder
    hp, m, b, gb, p64, bufs, O = _setup(cuda, preset, scale_stop=9.0)
    tf = O.model_forward(p64, bufs, hp, O.to_torch(b), None, training=False)
    a1, a2 = tf["alignment1"], tf["alignment2"]                      # [B, T', N] float64
    fa = (a1.float().to(cuda), a2.float().to(cuda))
    out = FreeRunningDecoder(m, forced_alignments=fa, feed="softmax").run(gb)
    ref = O.infer_free_running(p64, bufs, hp, O.to_torch(b), forced=(a1, a2), feed="softmax")
    assert out["steps"] == ref["steps"] == a1.shape[1]
    np.testing.assert_allclose(out["mel"].cpu().numpy(), ref["mel"].numpy(), atol=2e-5)
    np.testing.assert_allclose(out["stop"].cpu().numpy(), ref["stop"].numpy(), atol=2e-5)
    np.testing.assert_allclose(out["alignment1"].cpu().numpy(),
                               a1.permute(0, 2, 1).numpy(), atol=1e-7)


def test_model_fn_eval_forced_alignment_mode(cuda):
    """model_fn EVAL with use_forced_alignment_mode: the loss of the forced pass's outputs
    (0.1 * L1 + BCE, models/models.py:159-173) equals the oracle's on its restatement."""
    from sat_amd import hparams, models as MD, params
    from sat_amd.models import PreprocessedSourceData, PreprocessedTargetData
    from oracle import sat_oracle as O
    from sat_amd import data
    hp = hparams.ljspeech_hparams()
    hp.set_hparam("use_forced_alignment_mode", True)
    vals = params.init_params(hp, seed=5)
    model = MD.DualSourceSelfAttentionTacotronModel(hp, device=cuda, init_values=vals)
    b = data.synthetic_batch(hp, 2, N=11, T=16, shape="ljs", seed=4)
    ids = np.arange(2)
    feats = PreprocessedSourceData(ids, ids, b["source"], b["source_length"], None)
    labels = PreprocessedTargetData(ids, ids, b["mel"], b["target_length"], b["done"],
                                    b["mel_mask"], b["done_mask"])
    spec = model.model_fn(feats, labels, MD.ModeKeys.EVAL, hp)
    p64, bufs, tb = O.to_torch(vals), O.to_torch(params.init_bn_buffers(hp)), O.to_torch(b)
    tf = O.model_forward(p64, bufs, hp, tb, None, training=False)
    ref = O.infer_free_running(p64, bufs, hp, tb, forced=(tf["alignment1"], tf["alignment2"]),
                               feed="softmax")
    l = O.losses(ref["mel"], ref["stop"].unsqueeze(-1), tb["mel"], tb["mel_mask"], tb["done"],
                 tb["done_mask"])
    ref_loss = float(l["loss"]) if isinstance(l, dict) else float(l[0])
    assert abs(float(spec.loss.item()) - ref_loss) < 1e-5 * max(1.0, abs(ref_loss))


def _vbatch(cuda, preset="ljspeech", B=3, N=15, T=40, seed=6):
    from sat_amd import data, engine, hparams, params
    from oracle import sat_oracle as O
    hp = getattr(hparams, f"{preset}_hparams")()
    vals = params.init_params(hp, seed=5)
    m = engine.Tacotron(hp, cuda, init_values=vals)
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="ljs", seed=seed)
    gb = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
    return hp, vals, m, b, gb, O


@pytest.mark.parametrize("feed", ["softmax", "target"])
@pytest.mark.parametrize("preset", ["ljspeech", "vctk"])
def test_validation_decode_matches_oracle(cuda, preset, feed):
    """OneHotValidationHelper (modules/helpers.py:61-108): exactly T' steps with the real
    attention; feed = softmax of the previous output (teacher_forcing=False, EVAL's loss) or the
    target frame (teacher_forcing=True).  HIP vs the oracle's restatement."""
    from sat_amd import params
    from sat_amd.inference import FreeRunningDecoder
    hp, vals, m, b, gb, O = _vbatch(cuda, preset)
    out = FreeRunningDecoder(m, helper="validation", feed=feed).run(gb)
    ref = O.infer_free_running(O.to_torch(vals), O.to_torch(params.init_bn_buffers(hp)), hp,
                               O.to_torch(b), helper="validation", feed=feed)
    Tp = b["mel"].shape[1] // hp.outputs_per_step
    assert out["steps"] == ref["steps"] == Tp
    np.testing.assert_allclose(out["mel"].cpu().numpy(), ref["mel"].numpy(), atol=2e-5)
    np.testing.assert_allclose(out["stop"].cpu().numpy(), ref["stop"].numpy(), atol=2e-5)
    np.testing.assert_allclose(out["alignment1"].cpu().numpy(),
                               ref["alignment1"].permute(0, 2, 1).numpy(), atol=2e-6)


def test_model_fn_eval_losses_match_oracle(cuda):
    """model_fn EVAL (models/models.py:84-97, 151-173, 208-235, 305-320): ``loss`` /
    ``code_loss`` / ``done_loss`` from the softmax-fed validation decode, the ``*_with_teacher``
    metrics from the teacher-forced pass -- both vs the oracle."""
    from sat_amd import hparams, models as MD, params
    from sat_amd.models import PreprocessedSourceData, PreprocessedTargetData
    hp, vals, m, b, gb, O = _vbatch(cuda, B=2, N=12, T=24, seed=8)
    model = MD.DualSourceSelfAttentionTacotronModel(hp, device=cuda, init_values=vals)
    ids = np.arange(2)
    feats = PreprocessedSourceData(ids, ids, b["source"], b["source_length"], None)
    labels = PreprocessedTargetData(ids, ids, b["mel"], b["target_length"], b["done"],
                                    b["mel_mask"], b["done_mask"])
    spec = model.model_fn(feats, labels, MD.ModeKeys.EVAL, hp)
    p64, bufs, tb = O.to_torch(vals), O.to_torch(params.init_bn_buffers(hp)), O.to_torch(b)
    val = O.infer_free_running(p64, bufs, hp, tb, helper="validation", feed="softmax")
    loss, l1, bce = O.losses(val["mel"], val["stop"].unsqueeze(-1), tb["mel"], tb["mel_mask"],
                             tb["done"], tb["done_mask"])
    teach = O.model_forward(p64, bufs, hp, tb, None, training=False)
    mt = spec.eval_metric_ops
    close = lambda a, r: abs(float(a.item()) - float(r)) <= 1e-5 * max(1.0, abs(float(r)))  # noqa
    assert close(spec.loss, loss)
    assert close(mt["code_loss"], 0.1 * l1) and close(mt["done_loss"], bce)
    assert close(mt["loss_with_teacher"], teach["loss"])
    assert close(mt["code_loss_with_teacher"], 0.1 * teach["l1"])
    assert close(mt["done_loss_with_teacher"], teach["bce"])
    assert abs(float(spec.loss.item()) - float(mt["loss_with_teacher"].item())) > 1e-6


@pytest.mark.parametrize("B,N,T", [(3, 15, 40), (32, 200, 1000)], ids=["small", "c2_full"])
def test_teacher_forced_incremental_equals_training(cuda, B, N, T):
    """modules/transformer_test.py:44-90 on the HIP path: the training branch (teacher-forced
    dynamic_decode + causal self-attention over the whole output, here the persistent kernels
    and the batched head) equals the incremental branch driven by
    OneHotValidationHelper(teacher_forcing=True) (per-step kernels + TransformerWrapper's
    re-run, here the KV-cached head): outputs, stop tokens and argmax samples.  The two paths
    share no kernel of the decoder loop, so agreement is to fp32 rounding: mel max-abs <= 5e-5
    and mean-abs <= 2e-6 (the reference asserts rtol = atol = 1e-6 on TF's single path)."""
    from sat_amd.inference import FreeRunningDecoder
    hp, vals, m, b, gb, O = _vbatch(cuda, B=B, N=N, T=T, seed=9)
    with torch.no_grad():
        tr, _ = m.forward(gb, None, training=False, need_grad=False)
    inc = FreeRunningDecoder(m, helper="validation", feed="target").run(gb)
    d_mel = (tr["mel"] - inc["mel"]).abs()
    d_stop = (tr["stop"].view_as(inc["stop"]) - inc["stop"]).abs()
    r = hp.outputs_per_step
    s_tr = tr["mel"].view(B, -1, r, hp.num_mels).argmax(-1)
    s_in = inc["mel"].view(B, -1, r, hp.num_mels).argmax(-1)
    agree = float((s_tr == s_in).float().mean())
    path = os.environ.get("SAT_PARITY_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"case": f"a17_{B}x{N}x{T}", "mel_max_abs": float(d_mel.max()),
                                "mel_mean_abs": float(d_mel.mean()),
                                "stop_max_abs": float(d_stop.max()),
                                "sample_agreement": agree}) + "\n")
    assert float(d_mel.max()) <= 5e-5 and float(d_mel.mean()) <= 2e-6
    assert float(d_stop.max()) <= 5e-5
    assert agree >= 0.999                     # argmax ties may flip under rounding


def test_graph_decode_equals_eager(cuda):
    """Chunked hipGraph capture of the decode (graphs=True) replays the eager launches:
    bitwise-equal outputs, early stop included, and a second replay of the same plan."""
    from sat_amd.inference import FreeRunningDecoder
    hp, vals, m, b, gb, O = _vbatch(cuda, B=3, N=15, T=20, seed=2)
    eager = FreeRunningDecoder(m, max_iters=40, check_every=7).run(gb)
    dec = FreeRunningDecoder(m, max_iters=40, check_every=7, graphs=True)
    g1 = dec.run(gb)
    g2 = dec.run(gb)
    for g in (g1, g2):
        assert g["steps"] == eager["steps"]
        assert torch.equal(g["mel"], eager["mel"]) and torch.equal(g["stop"], eager["stop"])
        assert torch.equal(g["alignment1"], eager["alignment1"])
    val_e = FreeRunningDecoder(m, helper="validation", feed="softmax").run(gb)
    val_g = FreeRunningDecoder(m, helper="validation", feed="softmax", graphs=True,
                               check_every=5).run(gb)
    assert torch.equal(val_e["mel"], val_g["mel"])


# ---- C5 at its configured size (BASELINE configs[4]: LJSpeech, B=8, N=200, 500 free-running
#      decoder steps feeding back the predicted mel; modules/module.py:766-784,
#      predict_mel.py:36-75)
def _c5_batch(cuda, seed=55):
    """bench.py's C5 input: B=8 utterances of 200 chars (shape "max"), random-init weights"""
    from sat_amd import data, engine, hparams, params
    from oracle import sat_oracle as O
    hp = hparams.ljspeech_hparams()
    vals = params.init_params(hp, seed=5)
    m = engine.Tacotron(hp, cuda, init_values=vals)
    b = data.synthetic_batch(hp, 8, N=200, T=1000, shape="max", seed=seed)
    gb = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
    return hp, vals, m, b, gb, O


def test_c5_first_250_steps_match_oracle(cuda):
    """The first 250 free-running steps at B=8, N=200 (mel feedback, KV-cached head) vs the
    oracle's restatement (TransformerWrapper re-running the causal self-attention over the whole
    history each step).  The decode feeds its own fp32 output back, so the fp32-vs-float64
    difference could compound through the recurrence: mel within 1e-5 absolute (max) and 1e-6
    mean-abs over the 250 steps, alignments and stop logits within 1e-5 (achieved: 2.5e-7 /
    4.0e-8 / 1.1e-7, profiles/r03_parity_fullsize.jsonl)."""
    from sat_amd import params
    from sat_amd.inference import FreeRunningDecoder
    hp, vals, m, b, gb, O = _c5_batch(cuda)
    T = 250
    out = FreeRunningDecoder(m, max_iters=T, min_iters=T, check_every=25, graphs=True).run(gb)
    ref = O.infer_free_running(O.to_torch(vals), O.to_torch(params.init_bn_buffers(hp)), hp,
                               O.to_torch(b), max_iters=T, min_iters=T)
    assert out["steps"] == ref["steps"] == T
    d = np.abs(out["mel"].double().cpu().numpy() - ref["mel"].numpy())
    da = np.abs(out["alignment1"].double().cpu().numpy()
                - ref["alignment1"].permute(0, 2, 1).numpy())
    path = os.environ.get("SAT_PARITY_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"case": "c5_first250", "mel_max_abs": float(d.max()),
                                "mel_mean_abs": float(d.mean()),
                                "align1_max_abs": float(da.max())}) + "\n")
    assert float(d.max()) <= 1e-5 and float(d.mean()) <= 1e-6, (float(d.max()), float(d.mean()))
    assert float(da.max()) <= 1e-5
    np.testing.assert_allclose(out["stop"].cpu().numpy(), ref["stop"].numpy(), atol=1e-5)


def test_c5_full_length_closure(cuda):
    """All 500 free-running steps at B=8, N=200 closed on themselves: the teacher-forced
    training branch (persistent kernels, batched causal head) fed the decode's OWN predicted
    frames as targets reproduces those frames (TransformerTrainingHelper feeds
    targets[:, t-1, -80:], modules/helpers.py:54-58 -- exactly the frame the stop-token helper
    fed back).  Same bars as the A17 test: the two paths share no kernel of the loop."""
    from sat_amd.inference import FreeRunningDecoder
    hp, vals, m, b, gb, O = _c5_batch(cuda)
    T = 500
    fr = FreeRunningDecoder(m, max_iters=T, min_iters=T, check_every=25, graphs=True).run(gb)
    assert fr["steps"] == T and fr["mel"].shape == gb["mel"].shape
    tb = dict(gb)
    tb["mel"] = fr["mel"].contiguous()
    with torch.no_grad():
        tr, _ = m.forward(tb, None, training=False, need_grad=False)
    d_mel = (tr["mel"] - fr["mel"]).abs()
    d_stop = (tr["stop"].view_as(fr["stop"]) - fr["stop"]).abs()
    path = os.environ.get("SAT_PARITY_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"case": "c5_closure_500", "mel_max_abs": float(d_mel.max()),
                                "mel_mean_abs": float(d_mel.mean()),
                                "stop_max_abs": float(d_stop.max())}) + "\n")
    assert float(d_mel.max()) <= 5e-5 and float(d_mel.mean()) <= 2e-6
    assert float(d_stop.max()) <= 5e-5


def test_run_results_survive_the_next_run(cuda):
    """run() returns copies, never views of the per-shape plan's buffers: with B == 1 (where a
    reshape / contiguous of the step-major history would be a view), a second run on the same
    decoder and shape leaves the first result untouched."""
    from sat_amd.inference import FreeRunningDecoder
    hp, vals, m, b, gb, O = _vbatch(cuda, B=1, N=11, T=20, seed=12)
    dec = FreeRunningDecoder(m, max_iters=12, min_iters=12, check_every=4)
    r1 = dec.run(gb)
    mel1, stop1 = r1["mel"].clone(), r1["stop"].clone()
    gb2 = dict(gb)
    gb2["source"] = torch.flip(gb["source"], [1]).contiguous()   # a different utterance
    r2 = dec.run(gb2)
    assert not torch.equal(r2["mel"], mel1)
    assert torch.equal(r1["mel"], mel1) and torch.equal(r1["stop"], stop1)
