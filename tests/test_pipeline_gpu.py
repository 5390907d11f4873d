"""Chunked multi-stream schedule of the decoder recurrences (pipeline.Pipeline) == the
sequential schedule: outputs and every gradient, eager and hipGraph-captured."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(cuda, chunk, hp=None):
    from sat_amd import engine, hparams
    hp = hp or hparams.ljspeech_hparams()
    return engine.Tacotron(hp, cuda, seed=11, pipeline_chunk=chunk)


def _batch(cuda, hp, B=3, N=19, T=30, seed=4):
    from sat_amd import data
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="ljs", seed=seed)
    Np, Tp = b["source"].shape[1], b["mel"].shape[1] // hp.outputs_per_step
    m = data.synthetic_masks(hp, B, Np, Tp, seed=seed + 1)
    return ({k: torch.tensor(v).to(cuda) for k, v in b.items()},
            {k: torch.tensor(v).to(cuda) for k, v in m.items()})


@pytest.mark.parametrize("chunk", [1, 4, 6])
def test_pipelined_equals_sequential(cuda, chunk):
    seq = _model(cuda, 0)
    pip = _model(cuda, chunk)
    assert not seq.pipe.enabled and pip.pipe.enabled
    batch, masks = _batch(cuda, seq.hp)
    outs = []
    for m in (seq, pip):
        out, sv = m.forward(batch, masks, training=True)
        m.backward(sv)
        outs.append(out)
    torch.cuda.synchronize()
    assert float(outs[0]["loss"].item()) == pytest.approx(float(outs[1]["loss"].item()), rel=1e-6)
    np.testing.assert_allclose(outs[1]["mel"].cpu().numpy(), outs[0]["mel"].cpu().numpy(),
                               rtol=0, atol=1e-6)
    g0, g1 = seq.grads.cpu().numpy(), pip.grads.cpu().numpy()
    scale = np.abs(g0).max()
    assert np.abs(g1 - g0).max() <= 1e-5 * scale


def test_pipelined_graph_replay_equals_eager(cuda):
    from sat_amd import train
    a, b = _model(cuda, 4), _model(cuda, 4)
    batch, _ = _batch(cuda, a.hp, seed=8)
    Np, Tp = batch["source"].shape[1], batch["mel"].shape[1] // a.hp.outputs_per_step
    ta = train.Trainer(a, 3, Np, Tp, seed=5)
    tb = train.Trainer(b, 3, Np, Tp, seed=5)
    g = train.GraphedStep(ta, batch, warmup=1)
    tb.step(batch)
    for _ in range(3):
        g.replay()
        tb.step(batch)
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params), "multi-stream graph replay diverged from eager"
