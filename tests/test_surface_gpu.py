"""Plugin surface on the GPU: HIP-backed mechanisms from attention_mechanism_factory stepped
like TF AttentionMechanisms vs the oracle mechanisms, and model_fn TRAIN / EVAL."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["forward", "additive"])
def test_mechanism_steps_match_oracle(cuda, kind):
    from sat_amd import attentions as A
    from oracle import sat_oracle as O
    B, N, M, Q, units = 3, 45, 64, 48, (224 if kind == "forward" else 32)
    g = torch.Generator().manual_seed(3)
    memory = torch.randn(B, N, M, generator=g)
    lengths = torch.tensor([45, 30, 7])
    fn = A.attention_mechanism_factory(A.AttentionOptions(kind, units, 10, 5, False, False, False))
    mech = fn(memory.to(cuda), lengths.to(cuda), query_depth=Q, seed=9)
    p = {f"m/{k}": v.detach().cpu().double() for k, v in mech.variables.items()}
    ref = O.make_attention(kind, p, "m", memory.double(), lengths)
    state = mech.initial_state(B)
    rstate = ref.initial_state(B, N, torch.float64)
    for step in range(4):
        query = torch.randn(B, Q, generator=g)
        a, state = mech(query.to(cuda), state)
        ra, rstate = ref(query.double(), rstate)
        torch.cuda.synchronize()
        np.testing.assert_allclose(a.cpu().numpy(), ra.numpy(), atol=2e-6, rtol=1e-4,
                                   err_msg=f"step {step}")
        assert torch.all(a[1, 30:] == 0) and torch.all(a[2, 7:] == 0)   # masked memory


def test_model_fn_eval_matches_golden_and_train_learns(cuda):
    from sat_amd import hparams, models as M, params
    G = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                             "golden_model.npz"))
    hp = hparams.ljspeech_hparams()
    model = M.tacotron_model_factory(hp, None, None, device=cuda,
                                     init_values=params.init_params(hp, seed=5))
    b = {k[len("batch__"):]: G[k] for k in G.files if k.startswith("batch__")}
    ids = np.arange(b["source"].shape[0])
    feats = M.PreprocessedSourceData(ids, ids, b["source"], b["source_length"], None)
    labels = M.PreprocessedTargetData(ids, ids, b["mel"], b["target_length"], b["done"],
                                      b["mel_mask"], b["done_mask"])
    spec = model.model_fn(feats, labels, M.ModeKeys.EVAL, hp)
    # eval__loss of the golden file is the teacher-forced loss (loss_with_teacher)
    got = float(spec.eval_metric_ops["loss_with_teacher"].item())
    assert abs(got - float(G["eval__loss"])) < 1e-5
    losses = [float(model.model_fn(feats, labels, M.ModeKeys.TRAIN, hp).loss.item())
              for _ in range(8)]
    assert losses[-1] < losses[0]
    spec = model.model_fn(feats, None, M.ModeKeys.PREDICT, hp)
    pr = spec.predictions
    B = b["source"].shape[0]
    T = pr["mel"].shape[1]
    assert pr["mel"].shape == (B, T, hp.num_mels) and pr["codes"].shape == pr["mel"].shape
    assert torch.all(pr["codes"].sum(-1) == 1)                       # one-hot per frame
    assert pr["alignment"].shape == (B, b["source"].shape[1], T // hp.outputs_per_step)
    assert "alignment3" in pr and "alignment5" in pr


def test_model_fn_vctk_multi_speaker_records(cuda):
    """C4 through the estimator surface: VCTK SourceData (speaker_id) / MelData records
    (datasets/vctk/dataset.py:31-46) drive TRAIN and EVAL; a missing speaker_id raises."""
    from sat_amd import hparams, models as M
    hp = hparams.vctk_hparams()
    model = M.tacotron_model_factory(hp, None, None, device=cuda, seed=3)
    it = iter(M.synthetic_input_fn(hp, 3, N=14, T=20, shape="ljs", seed=2)())
    feats, labels = next(it)
    assert isinstance(feats, M.SourceData) and isinstance(labels, M.MelData)
    assert feats.speaker_id.min() >= 225 and feats.speaker_id.max() < 225 + 152
    spk0 = model.engine.P["speaker_embedding"].clone()
    ev0 = float(model.model_fn(feats, labels, M.ModeKeys.EVAL, hp).loss.item())
    spec = None
    for _ in range(4):
        spec = model.model_fn(feats, labels, M.ModeKeys.TRAIN, hp)
    assert int(spec.train_op.item()) == 4 and np.isfinite(float(spec.loss.item()))
    # Adam moved the rows of the batch's speakers and no other row
    moved = (model.engine.P["speaker_embedding"] != spk0).any(dim=1).cpu().numpy()
    assert set(np.nonzero(moved)[0]) == set(np.asarray(feats.speaker_id) - 225)
    ev1 = float(model.model_fn(feats, labels, M.ModeKeys.EVAL, hp).loss.item())
    assert np.isfinite(ev1) and ev1 != ev0
    with pytest.raises(ValueError):
        model.model_fn(feats._replace(speaker_id=None), labels, M.ModeKeys.EVAL, hp)
