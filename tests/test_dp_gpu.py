"""The data-parallel exchange's device half (C3; reference train.py:67-73 and the
cross-replica gradient aggregation of models/models.py:183-189) on the GPU box.

* ``sat_exchange_pack`` -> SUM over an emulated world of 8 replicas -> ``sat_exchange_unpack``
  on device arenas, bitwise against the host restatement that the gloo tests run
  (``dp.exchange``'s CPU branch): BN statistics pre-scaled by 1/8, health codes set on one or
  two "ranks" only.
* A ONE-rank ``nccl`` (= RCCL) process group opened in this process (127.0.0.1): the trainer
  forced through the full exchange (pack, the real RCCL all-reduce, unpack) between the two
  graphs of ``GraphedStep(split=True)`` replays bitwise like the unsplit single graph, since a
  one-rank SUM is the identity and 1/1 scaling is exact.
"""
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _host_exchange(arenas, healths, n_p, n_bn, n_h):
    """dp.exchange's host restatement over an emulated world (the same arithmetic, summed in
    rank order)."""
    w = len(arenas)
    packed = []
    for a, h in zip(arenas, healths):
        a = a.clone()
        a[n_p + n_bn:n_p + n_bn + n_h] = h.abs().float()
        a[n_p:n_p + n_bn] *= 1.0 / w
        packed.append(a)
    s = packed[0].clone()
    for a in packed[1:]:
        s += a
    return s, s[n_p + n_bn:n_p + n_bn + n_h].to(torch.int32)


def test_exchange_pack_unpack_matches_host_restatement(cuda):
    from sat_amd import _lib
    from sat_amd import kernels as K
    lib = _lib.load()
    g = torch.Generator().manual_seed(3)
    W, n_p, n_bn, n_h = 8, 100_003, 4_352, 16
    arenas = [torch.randn(n_p + n_bn + n_h, generator=g) for _ in range(W)]
    healths = [torch.zeros(n_h, dtype=torch.int32) for _ in range(W)]
    healths[3][0] = 1                 # one rank's attention-chain hand-off timeout
    healths[3][8] = -7                # a negative code travels as |code|
    healths[5][2] = 2
    healths[5][15] = (1 << 24) - 3    # largest exactly representable range
    ref_sum, ref_health = _host_exchange(arenas, healths, n_p, n_bn, n_h)

    dev = [a.to(cuda) for a in arenas]
    dh = [h.to(cuda) for h in healths]
    for a, h in zip(dev, dh):
        _lib.check(lib.sat_exchange_pack(h.data_ptr(), n_h, a[n_p:].data_ptr(), n_bn,
                                         a[n_p + n_bn:].data_ptr(), 1.0 / W, K._stream()),
                   "sat_exchange_pack")
    s = dev[0].clone()
    for a in dev[1:]:
        s += a                          # the all-reduce's SUM, in rank order
    out = []
    for a, h in zip(dev, dh):
        a.copy_(s)
        _lib.check(lib.sat_exchange_unpack(a[n_p + n_bn:].data_ptr(), n_h, h.data_ptr(),
                                           K._stream()), "sat_exchange_unpack")
        out.append(h)
    torch.cuda.synchronize()
    assert torch.equal(s.cpu(), ref_sum)
    for h in out:                       # every rank reads the same words back
        assert torch.equal(h.cpu(), ref_health)
    assert ref_health[0] == 1 and ref_health[8] == 7 and ref_health[2] == 2
    assert ref_health[15] == (1 << 24) - 3
    assert int((ref_health != 0).sum()) == 4


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_split_step_with_rccl_exchange_equals_unsplit(cuda):
    """GraphedStep(split=True) with the real RCCL all-reduce (one-rank nccl group, exchange
    forced) == the unsplit single graph, bitwise: parameters, Adam moments, BN statistics."""
    import torch.distributed as tdist
    from sat_amd import data, dp, engine, hparams, train
    if tdist.is_initialized():
        pytest.skip("a process group is already open in this process")
    tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                             world_size=1, device_id=cuda)
    try:
        hp = hparams.ljspeech_hparams()
        b = data.synthetic_batch(hp, 2, N=11, T=16, shape="ljs", seed=4)
        batch = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
        N, Tp = batch["source"].shape[1], batch["mel"].shape[1] // 2
        m1 = engine.Tacotron(hp, cuda, seed=42)
        m2 = engine.Tacotron(hp, cuda, seed=42)
        t1 = train.Trainer(m1, 2, N, Tp, seed=7)
        t2 = train.Trainer(m2, 2, N, Tp, seed=7, process_group=tdist.group.WORLD,
                           force_exchange=True)
        assert t2.world == 1 and t2.cfg.grad_scale == 1.0
        calls = []
        real = dp.tdist.all_reduce

        def counted(t, *a, **kw):
            calls.append(t.numel())
            return real(t, *a, **kw)

        dp.tdist.all_reduce = counted
        try:
            g1 = train.GraphedStep(t1, batch, warmup=1, split=False)
            g2 = train.GraphedStep(t2, batch, warmup=1, split=True)
            for _ in range(3):
                g1.replay()
                g2.replay()
            torch.cuda.synchronize()
        finally:
            dp.tdist.all_reduce = real
        assert calls == [m2.exchange.numel()] * (1 + 3)     # one collective per step
        t2.check_health(wait=True)
        assert torch.equal(m1.params, m2.params)
        assert torch.equal(t1.exp_avg, t2.exp_avg)
        assert torch.equal(t1.exp_avg_sq, t2.exp_avg_sq)
        assert torch.equal(m1.bn.buf, m2.bn.buf)
        assert int(t2.global_step.item()) == 4
        # the health tail went through pack -> RCCL -> unpack: |code| floats of a healthy step
        assert torch.equal(m2.health_tail[:m2.health.numel()],
                           torch.zeros(m2.health.numel(), device=cuda))
        # the bucketed exchange: the decoder's gradient rows all-reduced on a
        # comm stream once the decoder backward is issued -- captured INSIDE the forward /
        # backward graph, beside the encoder backward -- the rest between the two graphs;
        # bitwise the single-exchange step
        m3 = engine.Tacotron(hp, cuda, seed=42)
        t3 = train.Trainer(m3, 2, N, Tp, seed=7, process_group=tdist.group.WORLD,
                           force_exchange=True, bucketed=True)
        lo, hi = m3.decoder_grad_span()
        assert 0 < lo < hi == m3.params.numel() and lo % 64 == 0
        calls.clear()
        dp.tdist.all_reduce = counted
        try:
            g3 = train.GraphedStep(t3, batch, warmup=1, split=True)
            for _ in range(3):
                g3.replay()
            torch.cuda.synchronize()
        finally:
            dp.tdist.all_reduce = real
        rest = m3.exchange.numel() - hi
        # warm-up step (3 collectives), the captured bucket, then 2 eager ones per replay
        assert calls == [hi - lo, lo, rest, hi - lo] + [lo, rest] * 3
        t3.check_health(wait=True)
        assert torch.equal(m1.params, m3.params)
        assert torch.equal(t1.exp_avg, t3.exp_avg)
        assert torch.equal(t1.exp_avg_sq, t3.exp_avg_sq)
        assert torch.equal(m1.bn.buf, m3.bn.buf)
    finally:
        tdist.destroy_process_group()
