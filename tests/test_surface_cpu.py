"""Plugin surface without a GPU: AttentionOptions / factory dispatch and error behaviour
(modules/attentions.py:15-62, models/attention_factories.py:11-37, models/models.py:325-378)."""
import pytest
import torch

import _sat_path

_sat_path.load()
from sat_amd import attentions as A  # noqa: E402
from sat_amd import hparams, models as M  # noqa: E402


def test_attention_options_fields():
    assert A.AttentionOptions._fields == ("attention", "num_units", "attention_kernel",
                                          "attention_filters", "smoothing", "cumulative_weights",
                                          "use_transition_agent")


def test_dual_source_factory_reads_hparams():
    hp = hparams.ljspeech_hparams()
    f1, f2 = A.dual_source_attention_factory(hp)
    assert f1.options == A.AttentionOptions("forward", 224, 10, 5, False, False, False)
    assert f2.options == A.AttentionOptions("additive", 32, 10, 5, False, False, False)
    f = A.attention_factory(hp)
    assert f.options.num_units == hp.attention_out_units


def test_mechanism_dispatch_errors():
    unknown = A.attention_mechanism_factory(A.AttentionOptions("nope", 8, 3, 2, False, False, False))
    with pytest.raises(ValueError, match="Unknown attention mechanism"):
        unknown(None, None)
    fn = A.attention_mechanism_factory(A.AttentionOptions("location_sensitive", 8, 3, 2, False,
                                                          False, False))
    with pytest.raises(NotImplementedError):
        fn(None, None)
    for kind in ("teacher_forcing_forward", "teacher_forcing_additive"):
        fn = A.attention_mechanism_factory(A.AttentionOptions(kind, 8, 3, 2, False, False, False))
        with pytest.raises(TypeError, match="device tensor"):     # host memory is refused
            fn(torch.zeros(1, 2, 3), torch.ones(1, dtype=torch.int64), torch.zeros(1, 1, 2))


def test_force_alignment_factories_read_hparams():
    """models/attention_factories.py:40-66: the forced kinds come from
    forced_alignment_attention / forced_alignment_attention2 (hparams.py:95,99)."""
    hp = hparams.ljspeech_hparams()
    f1, f2 = A.force_alignment_dual_source_attention_factory(hp)
    assert f1.options == A.AttentionOptions("teacher_forcing_additive", 224, 10, 5, False, False,
                                            False)
    assert f2.options == A.AttentionOptions("teacher_forcing_additive", 32, 10, 5, False, False,
                                            False)
    assert A.force_alignment_attention_factory(hp).options.num_units == hp.attention_out_units


@pytest.mark.parametrize("field,factory", [("encoder", lambda hp: M.encoder_factory(hp, True)),
                                           ("decoder", M.decoder_factory),
                                           ("tacotron_model",
                                            lambda hp: M.tacotron_model_factory(hp, None, None))])
def test_model_factories_reject_unknown_names(field, factory):
    hp = hparams.ljspeech_hparams()
    hp.set_hparam(field, "NoSuchThing")
    with pytest.raises(ValueError, match="Unknown"):
        factory(hp)


def test_factories_build_from_reference_names():
    hp = hparams.ljspeech_hparams()
    enc = M.encoder_factory(hp, True)
    dec = M.decoder_factory(hp)
    assert enc.config["conv_channels"] == 128 and enc.config["max_filter_width"] == 16
    assert dec.config["outputs_per_step"] == 2 and dec.config["max_iters"] == 500


def test_learning_rate_decay_matches_reference_formula():
    f = M.DualSourceSelfAttentionTacotronModel.learning_rate_decay
    assert f(5e-4, 0, 1) == pytest.approx(5e-4 * 4000 ** 0.5 * 4000 ** -1.5)
    assert f(5e-4, 3999, 1) == pytest.approx(5e-4 * 4000 ** 0.5 * 4000 ** -0.5)
    assert f(5e-4, 15999, 1) == pytest.approx(5e-4 * 4000 ** 0.5 * 16000 ** -0.5)


def test_unbuilt_options_raise():
    """Options the reference accepts but this build does not compute raise instead of being
    silently ignored."""
    import types
    import pytest
    from sat_amd import hparams, params
    from sat_amd.inference import FreeRunningDecoder
    hp = hparams.ljspeech_hparams()
    hp.set_hparam("code_loss_type", "mse")
    with pytest.raises(NotImplementedError, match="code_loss_type"):
        params.resolve_dims(hp)
    hp = hparams.ljspeech_hparams()
    hp.set_hparam("use_l2_regularization", True)
    with pytest.raises(NotImplementedError, match="l2"):
        params.resolve_dims(hp)
    hp = hparams.ljspeech_hparams()
    hp.set_hparam("apply_dropout_on_inference", True)
    fake = types.SimpleNamespace(hp=hp, d=params.resolve_dims(hp))
    with pytest.raises(NotImplementedError, match="apply_dropout_on_inference"):
        FreeRunningDecoder(fake)
    hp = hparams.ljspeech_hparams()
    fake = types.SimpleNamespace(hp=hp, d=params.resolve_dims(hp))
    with pytest.raises(ValueError, match="validation helper"):
        FreeRunningDecoder(fake, feed="target")
    dec = FreeRunningDecoder(fake, helper="validation", feed="target")
    assert dec.helper == "validation" and dec.feed == "target"
