"""Host-side surface without a GPU: hparams (reference hparams.py / examples/*.json), the
parameter layout of the flat arena, mask and synthetic-batch contracts."""
import json
import os

import numpy as np
import pytest

import _sat_path

_sat_path.load()
from sat_amd import data, hparams, masks, params  # noqa: E402

REF = "/root/reference/examples"


@pytest.mark.parametrize("name,fn", [("ljspeech", hparams.ljspeech_hparams),
                                     ("vctk", hparams.vctk_hparams)])
def test_hparams_match_reference_json(name, fn):
    """create_hparams(json) == the preset (values read in place from the reference's example
    config when it is present -- this container only; the GPU box has no /root/reference)."""
    path = os.path.join(REF, name, "self-attention-tacotron.json")
    if not os.path.exists(path):
        pytest.skip("reference examples not present")
    hp = hparams.create_hparams(path)
    preset = fn()
    skip = {"average_mel_level_db", "stddev_mel_level_db"}  # denormalisation stats (off path)
    for k, v in json.load(open(path)).items():
        assert getattr(hp, k) == v
        if k not in skip:
            assert getattr(preset, k) == v, k


def test_hparams_parse_precedence_and_types():
    hp = hparams.create_hparams(overrides="outputs_per_step=3,attention=additive,"
                                          "decoder_prenet_out_units=[128,64]")
    assert hp.outputs_per_step == 3 and hp.attention == "additive"
    assert list(hp.decoder_prenet_out_units) == [128, 64]
    with pytest.raises(ValueError):
        hp.parse("no_such_hparam=1")
    hp.set_hparam("initial_learning_rate", 1)        # int -> float coercion like tf HParams
    assert isinstance(hp.initial_learning_rate, float)


def test_param_count_and_layout_roundtrip():
    hp = hparams.ljspeech_hparams()
    assert params.count_params(hp) == 6_227_928
    specs = params.param_specs(hp)
    lay = params.Layout(specs)
    vals = params.init_params(hp, seed=3)
    flat = lay.pack(vals)
    back = lay.unpack(flat)
    for k, v in vals.items():
        np.testing.assert_array_equal(back[k], v)
    # every tensor starts on a 256-byte boundary of the arena
    assert all(o % 64 == 0 for o in lay.offsets.values())


def test_lstm_gate_interleave_is_a_permutation():
    hp = hparams.ljspeech_hparams()
    vals = params.init_params(hp, seed=4)
    for name, v in vals.items():
        if params.is_lstm_param(name):
            iv = params.to_internal(name, v)
            np.testing.assert_array_equal(params.from_internal(name, iv), v)
            np.testing.assert_array_equal(np.sort(iv.reshape(-1)), np.sort(v.reshape(-1)))


def test_mask_specs_shapes_and_rates():
    hp = hparams.ljspeech_hparams()
    B, N, Tp = 3, 11, 7
    specs = {s.name: s for s in masks.mask_specs(hp, B, N, Tp)}
    assert specs["enc/prenet0"].shape == (B, N, hp.encoder_prenet_out_units[0])
    assert specs["dec/prenet0"].shape[:2] == (Tp, B)
    assert specs["dec/lstm0/zc"].kind == "zoneout"
    m = data.synthetic_masks(hp, B, N, Tp, seed=1)
    for k, s in specs.items():
        assert m[k].shape == tuple(s.shape)
        vals = np.unique(m[k])
        if s.kind == "zoneout":
            assert set(vals) <= {0.0, 1.0}
        else:
            on = 1.0 / (1.0 - s.rate)
            assert all(v == 0.0 or abs(v - on) < 1e-6 for v in vals.astype(np.float64))


@pytest.mark.parametrize("shape", ["max", "ljs"])
def test_synthetic_batch_contract(shape):
    hp = hparams.ljspeech_hparams()
    r = hp.outputs_per_step
    b = data.synthetic_batch(hp, 4, N=30, T=40, seed=2, shape=shape)
    B, N = b["source"].shape
    T = b["mel"].shape[1]
    assert T % r == 0 and b["done"].shape == (B, T // r)
    assert np.all(b["source_length"] <= N) and np.all(b["target_length"] <= T)
    for i in range(B):
        L = int(b["source_length"][i])
        assert np.all(b["source"][i, :L] >= 1) and np.all(b["source"][i, L:] == 0)
        tl = int(b["target_length"][i])
        assert np.all(b["mel_mask"][i, :tl] == 1) and np.all(b["mel_mask"][i, tl:] == 0)
    if shape == "max":
        assert np.all(b["source_length"] == N) and np.all(b["target_length"] == T)


def test_free_running_try_persistent_reports_why():
    """FreeRunningDecoder._try_persistent (the default decode's eligibility at run time): a
    library REFUSAL (SAT_ERR_UNSUPPORTED) is reported, so run() falls back to the per-step
    launches with a warning (inference.py); a raised error word (a hand-off timeout inside a
    launch that started) or any other library error is a hard error."""
    import torch
    from sat_amd import _lib
    from sat_amd.inference import FreeRunningDecoder

    class Plan:
        def __init__(self):
            self.err = torch.zeros(1, dtype=torch.int32)

    dec = FreeRunningDecoder.__new__(FreeRunningDecoder)

    def refused(pl, Tm):
        raise _lib.SatLibraryError("sat_decode_persistent: SAT_ERR_UNSUPPORTED",
                                   _lib.SAT_ERR_UNSUPPORTED)

    def broken(pl, Tm):
        raise _lib.SatLibraryError("sat_decode_persistent: launch failed", -2)

    dec._run_persistent = refused
    assert "UNSUPPORTED" in dec._try_persistent(Plan(), 5)
    dec._run_persistent = broken
    with pytest.raises(_lib.SatLibraryError, match="launch failed"):
        dec._try_persistent(Plan(), 5)
    dec._run_persistent = lambda pl, Tm: pl.err.fill_(1)
    with pytest.raises(_lib.SatLibraryError, match="timed out"):
        dec._try_persistent(Plan(), 5)
    dec._run_persistent = lambda pl, Tm: None
    assert dec._try_persistent(Plan(), 5) is None


def test_persistent_fallback_warns_once_with_reason():
    """a training shape the one-launch persistent decoder cannot take
    (here B=64 per GPU, and N=300 at B=32) warns once per shape, naming why, before the
    per-step launch path runs; eligible shapes and an explicit persistent=False stay silent."""
    import warnings
    from sat_amd import decoder
    d = params.resolve_dims(hparams.ljspeech_hparams())
    decoder._FALLBACK_WARNED.clear()
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert decoder.use_persistent(d, 32, 200)
        assert decoder.use_persistent(d, 8, 1024)
        assert not decoder.use_persistent(d, 64, 200, persistent=False)
        assert w == []
        assert not decoder.use_persistent(d, 64, 200)
        assert not decoder.use_persistent(d, 64, 200)            # once per shape
        assert not decoder.use_persistent(d, 32, 300)
    msgs = [str(x.message) for x in w if issubclass(x.category, decoder.PersistentFallbackWarning)]
    assert len(msgs) == 2
    assert "per-GPU batch 64" in msgs[0] and "B=32, N=300" in msgs[1]
    assert decoder.persistent_ineligible_reason(d, 32, 256) is None
