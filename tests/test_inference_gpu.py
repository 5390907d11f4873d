"""C5 free-running inference (BASELINE configs[4]) on libsat_hip vs the CPU oracle's restatement
of the PREDICT path (oracle.infer_free_running: StopTokenBasedInferenceHelper + TransformerWrapper
re-running the causal self-attention over the whole history; modules/module.py:766-784,
modules/rnn_wrappers.py:87-124, 188-214, helpers analog modules/helpers.py:111-160).

Tolerances: the decode feeds its own predictions back for up to max_iters steps, so fp32 vs
float64 drift compounds through the recurrence; mel frames within 2e-4 absolute over 40 steps."""
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
