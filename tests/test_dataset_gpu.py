"""Records -> pipeline -> model_fn on the GPU: an LJSpeech-format
TFRecord corpus (preprocess/ljspeech.py:23-45 records) read by the dataset pipeline
(datasets/ljspeech/dataset.py) feeds model_fn EVAL / TRAIN unchanged; the EVAL loss equals the
oracle's on the same padded batch (loss within 1e-5)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_tfrecord_batches_drive_model_fn(cuda, tmp_path):
    from sat_amd import datasets as D, hparams, models as MD, params, tfrecord as R
    from oracle import sat_oracle as O
    hp = hparams.ljspeech_hparams()
    hp.set_hparam("max_iters", 40)
    hp.set_hparam("average_mel_level_db", [0.5] * 80)
    hp.set_hparam("stddev_mel_level_db", [2.0] * 80)
    rng = np.random.default_rng(3)
    srcs, tgts = [], []
    for i, (T, N) in enumerate([(30, 9), (25, 7), (34, 11), (28, 8)]):
        s, t = str(tmp_path / f"{i}.s"), str(tmp_path / f"{i}.t")
        R.write_preprocessed_source_data(i, f"LJ{i}", rng.integers(1, 71, N), f"u{i}", s)
        R.write_preprocessed_target_data(i, f"LJ{i}", rng.standard_normal((T, 80)).astype(
            np.float32), t)
        srcs.append(s)
        tgts.append(t)
    batches = list(D.DatasetSource.create_from_tfrecord_files(srcs, tgts, hp)
                   .prepare_and_zip().filter_by_max_output_length().group_by_batch(2))
    assert len(batches) == 2
    vals = params.init_params(hp, seed=5)
    model = MD.DualSourceSelfAttentionTacotronModel(hp, device=cuda, init_values=vals)
    feats, labels = batches[0]
    spec = model.model_fn(feats, labels, MD.ModeKeys.EVAL, hp)
    tb = {"source": feats.source, "source_length": feats.source_length, "mel": labels.mel,
          "mel_mask": labels.spec_loss_mask, "done": labels.done,
          "done_mask": labels.binary_loss_mask, "target_length": labels.target_length}
    ref = O.model_forward(O.to_torch(vals), O.to_torch(params.init_bn_buffers(hp)), hp,
                          O.to_torch(tb), None, training=False)
    ref_loss = float(ref["loss"])
    got = float(spec.eval_metric_ops["loss_with_teacher"].item())
    assert abs(got - ref_loss) < 1e-5 * max(1.0, abs(ref_loss))
    out = model.model_fn(*batches[1], MD.ModeKeys.TRAIN, hp)
    assert np.isfinite(float(out.loss.item()))
