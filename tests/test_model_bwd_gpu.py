"""Hand-written HIP backward vs autograd of the CPU oracle (float64): every parameter gradient."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(cuda, train, B=3, N=17, T=24, shape="ljs", seed=0, hp_over=None, preset="ljspeech"):
    from sat_amd import hparams, params, data, engine
    from oracle import sat_oracle as O
    hp = getattr(hparams, f"{preset}_hparams")(**(hp_over or {}))
    vals = params.init_params(hp, seed=5)
    m = engine.Tacotron(hp, cuda, init_values=vals)
    batch = data.synthetic_batch(hp, B, N=N, T=T, shape=shape, seed=seed)
    Np, Tp = batch["source"].shape[1], batch["mel"].shape[1] // hp.outputs_per_step
    masks = data.synthetic_masks(hp, B, Np, Tp, seed=seed + 9) if train else None
    gb = {k: torch.tensor(v).to(cuda) for k, v in batch.items()}
    gm = None if masks is None else {k: torch.tensor(v).to(cuda) for k, v in masks.items()}
    out, sv = m.forward(gb, gm, training=train)
    m.backward(sv)
    torch.cuda.synchronize()
    grads = m.grads_dict()
    p64 = {k: v.requires_grad_(True) for k, v in O.to_torch(vals).items()}
    bufs = O.to_torch(params.init_bn_buffers(hp))
    ref = O.model_forward(p64, bufs, hp, O.to_torch(batch),
                          None if masks is None else O.to_torch(masks), training=train)
    ref["loss"].backward()
    return grads, p64, out, ref


def _compare(grads, p64, tol=2e-4):
    bad = []
    gmax = max(float(p.grad.abs().max()) for p in p64.values())
    for name, p in p64.items():
        g_ref = p.grad.numpy()
        g = grads[name].astype(np.float64)
        # floor: gradients that are identically zero in exact arithmetic (key-projection biases
        # under softmax shift invariance, conv biases in front of training-mode BatchNorm)
        scale = max(np.abs(g_ref).max(), 1e-4 * gmax)
        err = np.abs(g - g_ref).max() / scale
        if not np.isfinite(err) or err > tol:
            bad.append((name, float(err), float(scale)))
    return bad


@pytest.mark.parametrize("train", [False, True])
def test_all_parameter_gradients_match_oracle(cuda, train):
    grads, p64, out, ref = _run(cuda, train)
    assert abs(float(out["loss"].item()) - float(ref["loss"].detach())) < 1e-5
    bad = _compare(grads, p64)
    assert not bad, bad


def test_gradients_max_shape_full_lengths(cuda):
    grads, p64, out, ref = _run(cuda, True, B=2, N=40, T=48, shape="max", seed=3)
    bad = _compare(grads, p64)
    assert not bad, bad


@pytest.mark.parametrize("train", [False, True])
def test_vctk_multi_speaker_gradients_match_oracle(cuda, train):
    """C4: VCTK self-attention-tacotron.json -- speaker Embedding(152, 16, offset 225)
    (models/models.py:43-46) feeding MultiSpeakerPreNet (modules/multi_speaker_modules.py:27-32);
    the speaker embedding and projection gradients are covered by the same comparison."""
    grads, p64, out, ref = _run(cuda, train, B=4, N=15, T=20, seed=11, preset="vctk")
    assert "speaker_embedding" in p64 and "decoder/prenet0/speaker_projection/kernel" in p64
    assert abs(float(out["loss"].item()) - float(ref["loss"].detach())) < 1e-5
    np.testing.assert_allclose(out["mel"].cpu().numpy(), ref["mel"].detach().numpy(), atol=2e-5)
    bad = _compare(grads, p64)
    assert not bad, bad
    # only the rows of the speakers present in the batch receive gradient
    g = grads["speaker_embedding"]
    assert np.count_nonzero(np.abs(g).sum(1)) <= 4
