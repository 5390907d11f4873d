"""Optimiser step (clip + TF Adam + Noam lr) vs the oracle, graph replay == eager, loss goes down."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda, B=2, N=11, T=16, seed=0):
    from sat_amd import hparams, data, engine, train
    hp = hparams.ljspeech_hparams()
    m = engine.Tacotron(hp, cuda, seed=42)
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="ljs", seed=seed)
    batch = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
    tr = train.Trainer(m, B, batch["source"].shape[1], batch["mel"].shape[1] // 2, seed=7)
    return hp, m, batch, tr


def test_adam_step_matches_oracle(cuda):
    from oracle import sat_oracle as O
    hp, m, batch, tr = _setup(cuda)
    tr.forward_backward(batch)
    torch.cuda.synchronize()
    p0 = m.params_dict()
    g = m.grads_dict()
    tr.apply()
    torch.cuda.synchronize()
    p1 = m.params_dict()
    names = list(p0)
    grads, norm = O.clip_by_global_norm([torch.tensor(g[k], dtype=torch.float64) for k in names], 1.0)
    assert abs(float(tr.scalars[0]) - norm) / norm < 1e-5
    lr = O.learning_rate(hp.initial_learning_rate, 0)
    assert abs(float(tr.scalars[2]) - lr) / lr < 1e-6
    for k, gk in zip(names, grads):
        ref, _, _ = O.adam_tf(torch.tensor(p0[k], dtype=torch.float64), gk,
                              torch.zeros_like(gk), torch.zeros_like(gk), lr, 1)
        np.testing.assert_allclose(p1[k], ref.numpy(), rtol=0, atol=2e-6)
    assert int(tr.global_step.item()) == 1


def test_graph_replay_equals_eager_and_trains(cuda):
    from sat_amd import engine, train
    hp, m, batch, tr = _setup(cuda, seed=3)
    # eager twin with identical weights / seeds
    m2 = engine.Tacotron(hp, cuda, seed=42)
    tr2 = train.Trainer(m2, 2, batch["source"].shape[1], batch["mel"].shape[1] // 2, seed=7)
    g = train.GraphedStep(tr, batch, warmup=1)      # 1 eager step + capture
    tr2.step(batch)
    losses = []
    for _ in range(6):
        g.replay()
        tr2.step(batch)
        losses.append(float(tr.last_loss.item()))
    torch.cuda.synchronize()
    assert torch.equal(m.params, m2.params), "graph replay diverged from eager execution"
    assert losses[-1] < losses[0]
