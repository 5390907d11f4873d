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


def test_split_replay_equals_unsplit(cuda):
    """GraphedStep's data-parallel form (forward/backward graph, eager reduce_grads, clip+Adam
    graph; train.py) replays bitwise like the single-graph form.  The collective is the one
    seam: with world 1 it is the identity, so the two must agree exactly."""
    from sat_amd import engine, train
    hp, m, batch, tr = _setup(cuda, seed=4)
    m2 = engine.Tacotron(hp, cuda, seed=42)
    tr2 = train.Trainer(m2, 2, batch["source"].shape[1], batch["mel"].shape[1] // 2, seed=7)
    calls = []
    tr2.reduce_grads = lambda: calls.append(1)          # injected reducer (the RCCL seam)
    g1 = train.GraphedStep(tr, batch, warmup=1, split=False)
    g2 = train.GraphedStep(tr2, batch, warmup=1, split=True)
    assert g2.split and not g1.split
    for _ in range(3):
        g1.replay()
        g2.replay()
    torch.cuda.synchronize()
    assert len(calls) == 1 + 3                          # warm-up step + every replay
    assert torch.equal(m.params, m2.params)
    assert torch.equal(tr.exp_avg_sq, tr2.exp_avg_sq)


def test_health_guard_skips_update_and_raises(cuda):
    """a set error word of the step (here: the attention chain's hand-off timeout
    word, forced) makes the guarded Adam step skip the update on the device -- params, moments
    and global step untouched -- and the trainer raises at its next step without a sync."""
    from sat_amd import _lib
    hp, m, batch, tr = _setup(cuda, seed=5)
    tr.step(batch)
    torch.cuda.synchronize()
    tr.check_health(wait=True)                          # healthy step: no raise
    p0, gs0 = m.params.clone(), int(tr.global_step.item())
    tr.forward_backward(batch)
    m.health[0] = 1                                     # as a timed-out poll would leave it
    tr.apply()
    tr.publish_health()
    torch.cuda.synchronize()
    assert torch.equal(m.params, p0) and int(tr.global_step.item()) == gs0
    assert int(tr.status[0].item()) == 1 and int(tr.status[1].item()) == 1
    with pytest.raises(_lib.SatLibraryError, match="hand-off timeout"):
        tr.check_health(wait=True)


def test_model_fn_memory_flat_over_shapes(cuda):
    """model_fn TRAIN over many distinct padded shapes keeps one trainer (mask views
    re-pointed inside one arena) and one persistent scratch per batch size sized for the largest
    N -- device memory stays flat after the largest shape has been seen."""
    import gc
    from sat_amd import hparams, models as MD
    hp = hparams.ljspeech_hparams()
    # the eager drop-in path (graph_cache=0); the captured path keeps one graph pool per cached
    # shape, bounded by its LRU (test_model_fn_graph_cache_*)
    model = MD.DualSourceSelfAttentionTacotronModel(hp, device=cuda, seed=1, graph_cache=0)
    it = iter(MD.synthetic_input_fn(hp, 4, N=60, T=120, shape="ljs", seed=3)())
    feats, labels = next(it)
    big = MD.synthetic_input_fn(hp, 4, N=60, T=120, shape="max", seed=0)
    model.model_fn(*next(iter(big())), MD.ModeKeys.TRAIN, hp)      # the largest shape first
    torch.cuda.synchronize()
    gc.collect()
    base = torch.cuda.memory_allocated()
    shapes = set()
    for _ in range(12):
        f, l = next(it)
        shapes.add((f.source.shape[1], l.codes.shape[1]))
        model.model_fn(f, l, MD.ModeKeys.TRAIN, hp)
    torch.cuda.synchronize()
    gc.collect()
    assert len(shapes) >= 6
    assert torch.cuda.memory_allocated() <= base + (1 << 20)
    assert len(model.engine._scratch) == 1


def test_odd_rows_fused_attention_with_dropout(cuda):
    """B * N odd with T' % 4 == 0 and dropout on (advisor r5): every mask view starts on a
    16-byte boundary, so Python's and the library's fused-attention rules agree and the
    training step takes the fused path without a refusal; the step is finite and replays."""
    from sat_amd import train
    hp, m, batch, tr = _setup(cuda, B=1, N=13, T=16, seed=5)
    assert (batch["source"].shape[1] * 1) % 2 == 1 and (batch["mel"].shape[1] // 2) % 4 == 0
    tr.reshape(1, batch["source"].shape[1], batch["mel"].shape[1] // 2)
    assert all(v.data_ptr() % 16 == 0 for v in tr.masks.values())
    tr.forward_backward(batch)
    torch.cuda.synchronize()
    sv = tr.last_saved
    fused = [k for k, s in sv.items() if isinstance(s, dict) and s.get("lse") is not None]
    assert fused, "no multi-head attention took the fused path"
    assert np.isfinite(float(tr.last_loss.item()))
    assert torch.isfinite(m.grads).all()


def _shape_batches(hp, shapes, seed=0):
    from sat_amd import models as MD
    out = []
    for i, (B, N, T) in enumerate(shapes):
        it = iter(MD.synthetic_input_fn(hp, B, N=N, T=T, shape="max", seed=seed + 17 * i)())
        out.append(next(it))
    return out


def test_model_fn_graph_cache_equals_eager(cuda):
    """model_fn TRAIN replays one captured step per padded batch shape (LRU),
    eager only on a shape's first sighting; over two interleaved shapes the cached path's
    losses and parameters equal the eager drop-in path's bit for bit."""
    from sat_amd import hparams, models as MD
    hp = hparams.ljspeech_hparams()
    ma = MD.DualSourceSelfAttentionTacotronModel(hp, device=cuda, seed=3, graph_cache=4)
    mb = MD.DualSourceSelfAttentionTacotronModel(hp, device=cuda, seed=3, graph_cache=0)
    shapes = [(2, 13, 24), (2, 9, 32), (2, 13, 24), (2, 9, 32), (2, 13, 24), (2, 13, 24)]
    for f, l in _shape_batches(hp, shapes, seed=5):
        la = ma.model_fn(f, l, MD.ModeKeys.TRAIN, hp).loss
        lb = mb.model_fn(f, l, MD.ModeKeys.TRAIN, hp).loss
        torch.cuda.synchronize()
        assert torch.equal(la, lb)
        assert torch.equal(ma.engine.params, mb.engine.params)
    c = ma._graphs
    assert (c.misses, c.hits, c.evictions) == (2, 4, 0)
    assert int(ma._trainer.global_step.item()) == len(shapes)


def test_model_fn_graph_cache_lru_bound(cuda):
    """A cache of two graphs over three cycling shapes evicts the least recently used one each
    time; results stay equal to the eager path and the live graph count stays at the bound."""
    from sat_amd import hparams, models as MD
    hp = hparams.ljspeech_hparams()
    ma = MD.DualSourceSelfAttentionTacotronModel(hp, device=cuda, seed=4, graph_cache=2)
    mb = MD.DualSourceSelfAttentionTacotronModel(hp, device=cuda, seed=4, graph_cache=0)
    shapes = [(2, 11, 16), (2, 7, 24), (2, 11, 16), (2, 5, 20), (2, 7, 24), (2, 5, 20)]
    for f, l in _shape_batches(hp, shapes, seed=9):
        la = ma.model_fn(f, l, MD.ModeKeys.TRAIN, hp).loss
        lb = mb.model_fn(f, l, MD.ModeKeys.TRAIN, hp).loss
        torch.cuda.synchronize()
        assert torch.equal(la, lb)
    assert torch.equal(ma.engine.params, mb.engine.params)
    c = ma._graphs
    assert len(c.entries) == 2 and c.evictions == 2 and c.hits == 2


def test_graph_t_quantum_padding_keeps_the_step(cuda):
    """graph_t_quantum pads T' with the reference's own batch padding (mel -3.0, done 1, loss
    masks 0): with every dropout / zoneout rate 0 (so the masks are all ones and no draw can
    differ), the padded step's loss and gradients equal the unpadded step's to fp32 rounding."""
    from sat_amd import engine, hparams, train
    hp = hparams.ljspeech_hparams()
    for k in ("encoder_prenet_drop_rate", "decoder_prenet_drop_rate", "self_attention_drop_rate",
              "decoder_self_attention_drop_rate", "zoneout_factor_cell", "zoneout_factor_output"):
        hp.set_hparam(k, 0.0)
    (f, l), = _shape_batches(hp, [(2, 10, 22)], seed=2)
    from sat_amd import models as MD
    batch = MD.DualSourceSelfAttentionTacotronModel(hp, device=cuda, seed=1)._batch(f, l)
    res = []
    for q in (0, 8):
        m = engine.Tacotron(hp, cuda, seed=42)
        tr = train.Trainer(m, 2, batch["source"].shape[1], 16, seed=7)
        b = train.StepGraphCache(tr, 1, q)._pad_t(batch)
        assert b["mel"].shape[1] // 2 == (11 if q == 0 else 16)
        tr.reshape(2, b["source"].shape[1], b["mel"].shape[1] // 2)
        out = tr.forward_backward(b)
        torch.cuda.synchronize()
        res.append((float(out["loss"].item()), m.grads.clone()))
    (l0, g0), (l1, g1) = res
    assert abs(l0 - l1) <= 1e-6 * abs(l0)
    scale = float(g0.abs().max())
    assert float((g0 - g1).abs().max()) <= 2e-5 * scale
