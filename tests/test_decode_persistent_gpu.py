"""sat_decode_persistent (the whole free-running decode as ONE launch) against the per-step
launch path of the same FreeRunningDecoder (each of which is checked against the float64 oracle
in test_inference_gpu.py), and against the oracle directly.

The one-launch decode folds the fed frame into the first prenet layer and the value / output /
transform products into the cached rows (exact algebra, different fp32 rounding) and hands
LSB-tagged floats between workgroups (<= 1 ulp), so the paths agree to fp32 rounding through the
recurrence: mel within 2e-5 absolute over 40 steps, alignments within 2e-6, the decoder
self-alignment rows within 2e-6, the same step count (stop-token helper)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda, B, N, seed=2, stop_bias=None):
    from sat_amd import data, engine, hparams, params
    hp = hparams.ljspeech_hparams()
    vals = params.init_params(hp, seed=5)
    if stop_bias is not None:
        vals["decoder/stop_token_projection/bias"] = np.full((1,), stop_bias, np.float32)
    m = engine.Tacotron(hp, cuda, init_values=vals)
    b = data.synthetic_batch(hp, B, N=N, T=20, shape="ljs", seed=seed)
    gb = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
    return hp, vals, m, b, gb


def _both(m, gb, **kw):
    from sat_amd.inference import FreeRunningDecoder
    one = FreeRunningDecoder(m, persistent=True, **kw)
    ref = FreeRunningDecoder(m, persistent=False, **kw)
    a = one.run(gb)
    assert one.last_path == "persistent"
    b = ref.run(gb)
    assert ref.last_path == "launches"
    return a, b


@pytest.mark.parametrize("B,N", [(3, 15), (5, 40), (1, 7), (8, 200)])
def test_one_launch_matches_launch_path(cuda, B, N):
    hp, vals, m, b, gb = _setup(cuda, B, N)
    T = 40
    a, r = _both(m, gb, max_iters=T, min_iters=T)
    assert a["steps"] == r["steps"] == T
    dm = (a["mel"] - r["mel"]).abs()
    assert float(dm.max()) <= 2e-5, float(dm.max())
    assert float((a["stop"] - r["stop"]).abs().max()) <= 2e-5
    assert float((a["alignment1"] - r["alignment1"]).abs().max()) <= 2e-6
    assert float((a["alignment2"] - r["alignment2"]).abs().max()) <= 2e-6
    sa, sr = a["decoder_self_alignments"][0], r["decoder_self_alignments"][0]
    assert float((sa - sr).abs().max()) <= 2e-6


@pytest.mark.parametrize("bias", [8.0, -8.0])
def test_one_launch_stop_token(cuda, bias):
    """The in-kernel stop test (every group reads every utterance's stop granule) ends the
    decode at the same step as the launch path's stop_check latch."""
    hp, vals, m, b, gb = _setup(cuda, 3, 9, stop_bias=bias)
    a, r = _both(m, gb, max_iters=30, min_iters=10)
    assert a["steps"] == r["steps"] == (12 if bias > 0 else 30)
    assert float((a["mel"] - r["mel"]).abs().max()) <= 2e-5


def test_one_launch_matches_oracle(cuda):
    """Directly against the float64 oracle's PREDICT restatement (B=3, N=15, 40 steps): the
    test_inference_gpu.py bars."""
    from oracle import sat_oracle as O
    from sat_amd import params
    from sat_amd.inference import FreeRunningDecoder
    hp, vals, m, b, gb = _setup(cuda, 3, 15)
    T = 40
    dec = FreeRunningDecoder(m, max_iters=T, persistent=True)
    out = dec.run(gb)
    ref = O.infer_free_running(O.to_torch(vals), O.to_torch(params.init_bn_buffers(hp)), hp,
                               O.to_torch(b), max_iters=T)
    assert out["steps"] == ref["steps"]
    np.testing.assert_allclose(out["mel"].cpu().numpy(), ref["mel"].numpy(), atol=2e-4)
    np.testing.assert_allclose(out["alignment1"].cpu().numpy(),
                               ref["alignment1"].permute(0, 2, 1).numpy(), atol=2e-5)
    np.testing.assert_allclose(out["decoder_self_alignments"][0].cpu().numpy(),
                               ref["decoder_self_alignments"][0].numpy(), atol=2e-5)


def test_one_launch_rerun_is_deterministic(cuda):
    """Two decodes on the same plan (scratch re-cleared, caches rewritten) are bitwise equal."""
    from sat_amd.inference import FreeRunningDecoder
    hp, vals, m, b, gb = _setup(cuda, 4, 30)
    dec = FreeRunningDecoder(m, max_iters=64, min_iters=64, persistent=True)
    a = dec.run(gb)
    c = dec.run(gb)
    assert torch.equal(a["mel"], c["mel"]) and torch.equal(a["alignment1"], c["alignment1"])


def test_default_falls_back_when_one_launch_refused(cuda, monkeypatch):
    """persistent=None: when the library REFUSES the one-launch decode at run time
    (SAT_ERR_UNSUPPORTED, e.g. a device with too few co-resident workgroups) the run continues
    on the per-step launches from clean buffers with a warning and gives the launch path's
    result; a hand-off timeout inside a launch that started is a hard error (it
    would hide a regression), and persistent=True raises on a refusal too."""
    from sat_amd import _lib
    from sat_amd import kernels as K
    from sat_amd.inference import FreeRunningDecoder
    hp, vals, m, b, gb = _setup(cuda, 3, 15)
    T = 20
    ref = FreeRunningDecoder(m, persistent=False, max_iters=T, min_iters=T).run(gb)
    real = K.decode_persistent

    def refused(**kw):
        raise _lib.SatLibraryError("sat_decode_persistent: fewer than 256 co-resident workgroups",
                                   _lib.SAT_ERR_UNSUPPORTED)

    def timed_out(**kw):
        real(**kw)
        kw["err"].fill_(1)

    monkeypatch.setattr(K, "decode_persistent", timed_out)
    with pytest.raises(_lib.SatLibraryError, match="timed out"):
        FreeRunningDecoder(m, max_iters=T, min_iters=T).run(gb)
    for fake in (refused,):
        monkeypatch.setattr(K, "decode_persistent", fake)
        dec = FreeRunningDecoder(m, max_iters=T, min_iters=T)
        with pytest.warns(RuntimeWarning, match="falls back to per-step launches"):
            out = dec.run(gb)
        assert dec.last_path == "launches"
        assert out["steps"] == ref["steps"] == T
        assert torch.equal(out["mel"], ref["mel"])
        assert torch.equal(out["alignment1"], ref["alignment1"])
        out2 = dec.run(gb)                  # the plan stays on the launch path
        assert dec.last_path == "launches" and torch.equal(out2["mel"], ref["mel"])
        with pytest.raises(_lib.SatLibraryError):
            FreeRunningDecoder(m, persistent=True, max_iters=T, min_iters=T).run(gb)
