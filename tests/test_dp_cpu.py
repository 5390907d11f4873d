"""N>1 data-parallel path under ``gloo`` (world_size 2, and 8 = C3's rank count, CPU): the same
dp.py functions and Trainer.reduce_grads the bench runs over RCCL on the GPUs."""
import os
import socket
import types

import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import _sat_path
        _sat_path.load()
        from sat_amd import dp, hparams, train
        tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                 world_size=world)
        res = {}
        # broadcast of the parameter arena: every replica starts from rank 0's weights
        p = torch.full((1000,), float(rank + 1))
        dp.broadcast_params(p)
        res["bcast"] = bool(torch.all(p == 1.0))
        # every rank holds DIFFERENT local gradients, BN buffers and health words; the
        # exchange must leave each rank with the global-batch state
        hp = hparams.ljspeech_hparams()
        n = 4096

        def local_grad(r):
            g = torch.Generator().manual_seed(100 + r)
            return torch.randn(n, generator=g) * (1e-4 * (0.5 + r))   # global norm < clip_norm

        def local_bn(r):
            return torch.linspace(-1.0, 1.0, 64) * (r + 1) + 0.25 * r

        # the engine's exchange arena layout: [gradients | BN statistics | health tail]
        arena = torch.cat([local_grad(rank), local_bn(rank), torch.zeros(16)])
        model = types.SimpleNamespace(
            hp=hp, device=torch.device("cpu"), params=torch.zeros(n), exchange=arena,
            grads=arena[:n], health_tail=arena[n + 64:],
            health=torch.zeros(16, dtype=torch.int32),
            bn=types.SimpleNamespace(buf=arena[n:n + 64]))
        if rank == 1:
            model.health[3] = 7          # a hand-off timeout on rank 1 only
        tr = train.Trainer(model, B=2, N=8, Tp=4)
        calls = []
        real = tdist.all_reduce

        def counting(*a, **k):
            calls.append(a[0].numel())
            return real(*a, **k)

        tdist.all_reduce = counting
        tr.reduce_grads()
        tdist.all_reduce = real
        res["collectives"] = list(calls)
        gsum = sum(local_grad(r) for r in range(world))
        # world 2: a two-term sum is the same in any order (bitwise); at world 8 the backend's
        # reduction order differs from rank order in the last bits
        res["sum_err"] = float((model.grads - gsum).abs().max())
        res["sum"] = bool(torch.equal(model.grads, gsum)) if world == 2 else \
            bool(torch.allclose(model.grads, gsum, rtol=1e-6, atol=1e-9))
        res["scale"] = tr.cfg.grad_scale
        res["world"] = tr.world
        # BatchNorm moving statistics: the mean of the replicas' buffers
        bn_mean = sum(local_bn(r) for r in range(world)) / world
        res["bn"] = bool(torch.allclose(model.bn.buf, bn_mean, rtol=0, atol=1e-6))
        # health words combined by MAX: every rank sees rank 1's error, so the guarded update
        # is skipped everywhere (not applied on rank 0 and skipped on rank 1)
        res["health"] = model.health.tolist()
        # the optimiser on the reduced arena (host restatement of the fused clip + Adam step,
        # gradient scaled by cfg.grad_scale) == ONE process stepping on the global-batch mean
        # gradient; and the replicas agree
        from oracle import sat_oracle as O

        def adam_steps(g_fn):
            p = torch.linspace(-1, 1, n, dtype=torch.float64)
            mo = torch.zeros_like(p)
            vo = torch.zeros_like(p)
            for step in range(1, 3):
                (g,), _ = O.clip_by_global_norm([g_fn()], 1.0)
                p, mo, vo = O.adam_tf(p, g, mo, vo,
                                      O.learning_rate(hp.initial_learning_rate, step - 1), step)
            return p

        p_dp = adam_steps(lambda: model.grads.double() * tr.cfg.grad_scale)
        p_one = adam_steps(lambda: sum(local_grad(r).double() for r in range(world)) / world)
        # (world 8: the fp32 collective's summation order shows in the last bits of the update)
        res["matches_single"] = bool(torch.allclose(p_dp, p_one, rtol=0,
                                                    atol=1e-12 if world == 2 else 1e-9))
        gathered = [torch.empty_like(p_dp) for _ in range(world)]
        tdist.all_gather(gathered, p_dp)
        res["replicas_equal"] = all(torch.equal(gathered[0], x) for x in gathered[1:])
        # the bucketed exchange: the decoder rows [lo, hi) reduced first (the
        # hook model_backward calls once the decoder backward is issued), the rest at the end
        # -- bitwise the single exchange's result, in three collectives
        lo = 1024

        def fresh_model():
            a = torch.cat([local_grad(rank), local_bn(rank), torch.zeros(16)])
            mm = types.SimpleNamespace(
                hp=hp, device=torch.device("cpu"), params=torch.zeros(n), exchange=a,
                grads=a[:n], health_tail=a[n + 64:], health=torch.zeros(16, dtype=torch.int32),
                bn=types.SimpleNamespace(buf=a[n:n + 64]),
                decoder_grad_span=lambda: (lo, n))
            if rank == 1:
                mm.health[5] = 3
            return mm
        m1, m2 = fresh_model(), fresh_model()
        t1 = train.Trainer(m1, B=2, N=8, Tp=4, bucketed=False)
        t2 = train.Trainer(m2, B=2, N=8, Tp=4, bucketed=True)
        t1.reduce_grads()
        assert t2._bucketing()
        calls.clear()
        tdist.all_reduce = counting
        t2._decoder_bucket([])
        t2.reduce_grads()
        tdist.all_reduce = real
        res["bucket_collectives"] = list(calls)
        # bitwise at world 2; at world 8 the ring's per-chunk summation order depends on the
        # collective's length, so the bucketed ranges may differ from the single one in the
        # last bits (dp.exchange); health words are exact either way
        same = torch.equal if world == 2 else \
            (lambda a, b: torch.allclose(a, b, rtol=1e-6, atol=1e-9))
        res["bucket_equal"] = bool(same(m1.exchange, m2.exchange)) and \
            bool(torch.equal(m1.health, m2.health))
        # masks are drawn per replica: the model_fn seed offset differs by rank
        res["seed_offset"] = 1000003 * dp.rank()
        # max-over-ranks step time
        res["max"] = dp.max_over_ranks(0.5 + rank, "cpu")
        tdist.barrier()
        tdist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 8])
def test_dp_world_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        res = out[r]
        assert isinstance(res, dict), res
        assert res["sum"], res["sum_err"]
        assert res["bcast"] and res["sum"] and res["bn"] and res["replicas_equal"], res
        assert res["matches_single"]
        assert res["health"][3] == 7 and sum(res["health"]) == 7
        assert res["collectives"] == [4096 + 64 + 16]     # ONE collective per step
        assert res["bucket_equal"]
        assert res["bucket_collectives"] == [4096 - 1024, 1024, 64 + 16]
        assert res["seed_offset"] == 1000003 * r
        assert res["scale"] == pytest.approx(1.0 / world) and res["world"] == world
        assert res["max"] == pytest.approx(0.5 + world - 1)


def test_single_process_is_identity():
    import _sat_path
    _sat_path.load()
    from sat_amd import dp
    g = torch.ones(8)
    dp.allreduce_grads(g)
    assert torch.equal(g, torch.ones(8))
    assert dp.grad_scale() == 1.0 and dp.world_size() == 1
    assert dp.max_over_ranks(3.0, "cpu") == 3.0
