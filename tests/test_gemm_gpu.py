"""fp32 MFMA GEMM (sat_gemm) against torch fp64 CPU products, every operand mode."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double().cpu() - b.double()).abs().max() / (b.double().abs().max() + 1e-12))


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (33, 17, 5), (64, 64, 64), (200, 300, 129),
                                   (1000, 1024, 544), (6400, 128, 2048)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True)])
def test_gemm_dense(cuda, M, N, K, ta, tb):
    from sat_amd import kernels
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(K, M, generator=g) if ta else torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g) if tb else torch.randn(K, N, generator=g)
    bias = torch.randn(N, generator=g)
    Ad, Bd = A.to(cuda), B.to(cuda)
    C = kernels.gemm(Ad.t() if ta else Ad, Bd.t() if tb else Bd, bias=bias.to(cuda), act="tanh")
    Al, Bl = (A.t() if ta else A).double(), (B.t() if tb else B).double()
    ref = torch.tanh(Al @ Bl + bias.double())
    # fp32 accumulation bound (tanh is 1-Lipschitz): |err| <= c * eps32 * (|A| @ |B| + |bias|)
    bound = 4e-7 * (Al.abs() @ Bl.abs() + bias.double().abs()) + 1e-7
    assert bool(((C.double().cpu() - ref).abs() <= bound).all())


def test_gemm_batched_beta(cuda):
    from sat_amd import kernels
    g = torch.Generator().manual_seed(0)
    A, B, C0 = torch.randn(4, 50, 70, generator=g), torch.randn(4, 70, 30, generator=g), \
        torch.randn(4, 50, 30, generator=g)
    C = C0.to(cuda)
    kernels.gemm(A.to(cuda), B.to(cuda), C, alpha=0.5, beta=2.0)
    ref = 0.5 * A.double() @ B.double() + 2.0 * C0.double()
    assert _rel(C, ref) < 1e-5


def _conv_ref(x, W, b=None):
    from oracle.sat_oracle import conv1d_same
    return conv1d_same(x.double(), W.double(), None if b is None else b.double())


@pytest.mark.parametrize("taps", [1, 2, 3, 10, 16])
def test_conv1d_fwd_dx_dw(cuda, taps):
    from sat_amd import kernels
    g = torch.Generator().manual_seed(taps)
    S, L, Ci, Co = 3, 37, 24, 20
    x = torch.randn(S, L, Ci, generator=g, dtype=torch.float64, requires_grad=True)
    W = torch.randn(taps, Ci, Co, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(Co, generator=g, dtype=torch.float64)
    y = _conv_ref(x, W, b)
    dy = torch.randn(S, L, Co, generator=g, dtype=torch.float64)
    y.backward(dy)
    xd, Wd = x.detach().float().to(cuda), W.detach().float().to(cuda)
    yd = kernels.conv1d(xd, Wd, b.float().to(cuda))
    assert _rel(yd, y.detach()) < 1e-5
    dxd = kernels.conv1d_dx(dy.float().to(cuda), Wd)
    assert _rel(dxd, x.grad) < 1e-5
    dWd = torch.empty_like(Wd)
    kernels.conv1d_dw(xd, dy.float().to(cuda), dWd)
    assert _rel(dWd, W.grad) < 1e-5


def test_rng_fill(cuda):
    from sat_amd import kernels
    seed = torch.tensor([1234], dtype=torch.int64, device=cuda)
    out = torch.empty(1_000_003, device=cuda)
    kernels.rng_fill(out, seed, 7, 0.9, 1.0 / 0.9)
    vals = out.cpu()
    keep = float((vals != 0).double().mean())
    assert abs(keep - 0.9) < 3e-3
    assert torch.allclose(vals[vals != 0], torch.tensor(1.0 / 0.9))
    out2 = torch.empty_like(out)
    kernels.rng_fill(out2, seed, 7, 0.9, 1.0 / 0.9)
    assert torch.equal(out, out2)
    kernels.rng_fill(out2, seed, 8, 0.9, 1.0 / 0.9)
    assert not torch.equal(out, out2)


# ---- the LDS-DMA kernel (gemm_lds_kernel): every operand mode, ragged tile edges, split-K.
# Shapes follow the training step's products (SURVEY 8(d) census) at reduced M where possible.
@pytest.mark.parametrize("M,N,K", [(16000, 256, 256), (300, 1024, 288), (96, 160, 2000),
                                   (256, 1024, 16000), (544, 1024, 3000), (128, 4, 6400),
                                   (4, 128, 64), (130, 68, 36)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_lds_modes(cuda, M, N, K, ta, tb):
    from sat_amd import kernels
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(K, M, generator=g) if ta else torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g) if tb else torch.randn(K, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    C = C0.to(cuda)
    Ad, Bd = A.to(cuda), B.to(cuda)
    kernels.gemm(Ad.t() if ta else Ad, Bd.t() if tb else Bd, C, alpha=0.75, beta=0.5)
    Al, Bl = (A.t() if ta else A).double(), (B.t() if tb else B).double()
    ref = 0.75 * (Al @ Bl) + 0.5 * C0.double()
    bound = 6e-7 * (Al.abs() @ Bl.abs() + C0.double().abs()) + 1e-7
    err = (C.double().cpu() - ref).abs()
    assert bool((err <= bound).all()), float((err / bound).max())


@pytest.mark.parametrize("taps,Ci,Co,L", [(1, 128, 128, 100), (3, 128, 128, 77), (8, 128, 128, 200),
                                          (16, 128, 128, 60), (3, 2048, 128, 50), (3, 128, 64, 33)])
def test_conv1d_lds_fwd_dx_dw(cuda, taps, Ci, Co, L):
    from sat_amd import kernels
    g = torch.Generator().manual_seed(taps * 131 + L)
    S = 3
    x = torch.randn(S, L, Ci, generator=g, dtype=torch.float64, requires_grad=True)
    W = torch.randn(taps, Ci, Co, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(Co, generator=g, dtype=torch.float64)
    y = _conv_ref(x, W, b)
    dy = torch.randn(S, L, Co, generator=g, dtype=torch.float64)
    y.backward(dy)
    xd, Wd = x.detach().float().to(cuda), W.detach().float().to(cuda)
    yd = kernels.conv1d(xd, Wd, b.float().to(cuda))
    assert _rel(yd, y.detach()) < 2e-6
    dxd = kernels.conv1d_dx(dy.float().to(cuda), Wd)
    assert _rel(dxd, x.grad) < 2e-6
    dWd = torch.empty_like(Wd)
    kernels.conv1d_dw(xd, dy.float().to(cuda), dWd)
    assert _rel(dWd, W.grad) < 2e-6


@pytest.mark.parametrize("max_k,C,Co,S,L", [(16, 128, 128, 3, 37), (4, 64, 128, 2, 70),
                                            (5, 128, 64, 4, 9), (16, 128, 128, 32, 200)])
def test_conv_bank_matches_per_conv_oracle(cuda, max_k, C, Co, S, L):
    """sat_cbhg_convbank_fwd/bwd (one launch per direction) vs the float64 oracle Conv1D of each
    kernel width (ext tacotron2 Conv1d, modules/module.py:77-80)."""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(max_k * 7 + L)
    x = torch.randn(S, L, C, generator=g, dtype=torch.float64, requires_grad=True)
    Ws = [torch.randn(k, C, Co, generator=g, dtype=torch.float64, requires_grad=True) * 0.1
          for k in range(1, max_k + 1)]
    Ws = [w.detach().requires_grad_(True) for w in Ws]
    b = torch.randn(max_k * Co, generator=g, dtype=torch.float64)
    y = torch.cat([_conv_ref(x, Ws[k], b[k * Co:(k + 1) * Co]) for k in range(max_k)], dim=-1)
    dy = torch.randn(S, L, max_k * Co, generator=g, dtype=torch.float64)
    y.backward(dy)
    Wb = torch.cat([w.detach().reshape(-1) for w in Ws]).float().to(cuda)
    xd = x.detach().float().to(cuda)
    yd = torch.empty(S, L, max_k * Co, device=cuda)
    kernels.conv_bank(xd, Wb, b.float().to(cuda), yd, max_k, Co)
    assert _rel(yd, y.detach()) < 2e-6
    dx0 = torch.randn(S, L, C, generator=g)
    dxd = dx0.to(cuda)
    dW0 = torch.randn(Wb.numel(), generator=g)
    dWd = dW0.to(cuda)
    kernels.conv_bank_bwd(xd, Wb, dy.float().to(cuda), max_k, Co, dx=dxd, dW=dWd,
                          beta_dx=1.0, beta_dw=1.0)
    assert _rel(dxd, x.grad + dx0.double()) < 2e-6
    dW_ref = torch.cat([w.grad.reshape(-1) for w in Ws]) + dW0.double()
    assert _rel(dWd, dW_ref) < 2e-6
    # the training step's split calls (dW alone beside dX on another stream: at the C2 shape
    # the dW-only call takes its own measured plan, 128 x 128 tiles split 2)
    dWs = dW0.to(cuda)
    kernels.conv_bank_bwd(xd, Wb, dy.float().to(cuda), max_k, Co, dW=dWs, beta_dw=1.0)
    assert _rel(dWs, dW_ref) < 2e-6
    dxs = dx0.to(cuda)
    kernels.conv_bank_bwd(xd, Wb, dy.float().to(cuda), max_k, Co, dx=dxs, beta_dx=1.0)
    assert torch.equal(dxs, dxd)


@pytest.mark.parametrize("s", [1, 4])
def test_conv_bank_dx_large_tile(cuda, s):
    """The bank's input gradient (GRP 2) on the 256 x 128 tile (2-stage ring), forced, and on the
    cost model's plan, both against the float64 per-conv gradient (a 17,408-term fp32 reduction:
    1e-5 of the largest element)."""
    from sat_amd import _lib, kernels
    g = torch.Generator().manual_seed(77 + s)
    max_k, C, Co, S, L = 16, 128, 128, 4, 150
    x = torch.randn(S, L, C, generator=g, dtype=torch.float64, requires_grad=True)
    Ws = [(torch.randn(k, C, Co, generator=g, dtype=torch.float64) * 0.05).requires_grad_(True)
          for k in range(1, max_k + 1)]
    y = torch.cat([_conv_ref(x, Ws[k], torch.zeros(Co, dtype=torch.float64))
                   for k in range(max_k)], dim=-1)
    dy = torch.randn(S, L, max_k * Co, generator=g, dtype=torch.float64)
    y.backward(dy)
    Wd = torch.cat([w.detach().reshape(-1) for w in Ws]).float().to(cuda)
    xd, dyd = x.detach().float().to(cuda), dy.float().to(cuda)
    ref = torch.zeros(S, L, C, device=cuda)
    kernels.conv_bank_bwd(xd, Wd, dyd, max_k, Co, dx=ref, beta_dx=0.0)
    lib = _lib.load()
    out = torch.zeros(S, L, C, device=cuda)
    lib.sat_gemm_force_plan(256, 128, s)
    try:
        kernels.conv_bank_bwd(xd, Wd, dyd, max_k, Co, dx=out, beta_dx=0.0)
        torch.cuda.synchronize()
    finally:
        lib.sat_gemm_force_plan(0, 0, 0)
    assert _rel(ref, x.grad) < 1e-5
    assert _rel(out, x.grad) < 1e-5


# ---- forced plans: every tile shape incl. the 8-wave 128 x 128 variant, with and without split-K
@pytest.mark.parametrize("bm,bn,s", [(128, 128, 1), (128, 128, 4), (128, 64, 2), (64, 128, 1),
                                     (64, 64, 3), (256, 128, 1), (256, 128, 3), (128, 256, 1),
                                     (128, 256, 2)])
@pytest.mark.parametrize("M,N,K", [(1000, 520, 2048), (130, 260, 1024), (300, 200, 64),
                                   (257, 129, 96), (70, 300, 32)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_lds_forced_plans(cuda, bm, bn, s, M, N, K, ta, tb):
    from sat_amd import _lib, kernels
    g = torch.Generator().manual_seed(M + 5 * N + 11 * K + bm + s)
    A = torch.randn(K, M, generator=g) if ta else torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g) if tb else torch.randn(K, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    C = C0.to(cuda)
    Ad, Bd = A.to(cuda), B.to(cuda)
    lib = _lib.load()
    lib.sat_gemm_force_plan(bm, bn, s)
    try:
        kernels.gemm(Ad.t() if ta else Ad, Bd.t() if tb else Bd, C, alpha=1.25, beta=0.5)
        torch.cuda.synchronize()
    finally:
        lib.sat_gemm_force_plan(0, 0, 0)
    Al, Bl = (A.t() if ta else A).double(), (B.t() if tb else B).double()
    ref = 1.25 * (Al @ Bl) + 0.5 * C0.double()
    bound = 6e-7 * (Al.abs() @ Bl.abs() + C0.double().abs()) + 1e-7
    err = (C.double().cpu() - ref).abs()
    assert bool((err <= bound).all()), float((err / bound).max())


@pytest.mark.parametrize("bm,bn", [(128, 128), (64, 64), (256, 128), (128, 256)])
def test_conv1d_forced_plans(cuda, bm, bn):
    from sat_amd import _lib, kernels
    g = torch.Generator().manual_seed(bm + bn)
    x = torch.randn(6, 50, 128, generator=g)
    W = torch.randn(5, 128, 256, generator=g)
    lib = _lib.load()
    lib.sat_gemm_force_plan(bm, bn, 1)
    try:
        y = kernels.conv1d(x.to(cuda), W.to(cuda)).cpu().double()
        torch.cuda.synchronize()
    finally:
        lib.sat_gemm_force_plan(0, 0, 0)
    xp = torch.nn.functional.pad(x.double().transpose(1, 2), (2, 2))
    ref = torch.nn.functional.conv1d(xp, W.double().permute(2, 1, 0)).transpose(1, 2)
    assert float((y - ref).abs().max()) <= 2e-4 * float(ref.abs().max())


def test_rng_fill_segments_equals_per_mask_fills(cuda):
    """sat_rng_fill_segments (the step's masks in one launch) draws, per segment, exactly what
    sat_rng_fill draws on that segment's view with the same stream id."""
    from sat_amd import kernels
    sizes = [(5, 0.5, 2.0), (1000, 0.9, 1.0), (4097, 0.1, 10.0), (0, 0.5, 2.0), (64, 0.7, 1.0)]
    total = sum(n for n, _, _ in sizes) + 7
    seed = torch.tensor([0x1234_5678_9abc], dtype=torch.int64, device=cuda)
    base = torch.full((total,), -1.0, device=cuda)
    segs, off = [], 3
    for i, (n, keep, on) in enumerate(sizes):
        segs.append((off, n, 11 + i, keep, on))
        off += n
    end = off
    kernels.rng_fill_segments(base, kernels.rng_segments(segs), seed)
    for o, n, sid, keep, on in segs:
        ref = torch.empty(max(n, 1), device=cuda)[:n]
        if n:
            kernels.rng_fill(ref, seed, sid, keep, on)
        assert torch.equal(base[o:o + n], ref)
    assert float(base[:3].max()) == -1.0 and float(base[end:].max()) == -1.0   # untouched


# ---- fused column sums (SatGemmDesc.colsum_out): dW += X^T dY and db += colsum(dY) in one launch
@pytest.mark.parametrize("M,N,K", [(256, 1024, 3000), (128, 260, 500), (36, 64, 7000), (6, 40, 50)])
@pytest.mark.parametrize("ta", [True, False])
@pytest.mark.parametrize("split", [0, 4])
@pytest.mark.parametrize("alpha", [1.0, -0.75])
def test_gemm_colsum_fused(cuda, M, N, K, ta, split, alpha):
    """alpha applies to the product AND the column sums, on the fused LDS path and on the
    separate-reduction fallback (M % 4 != 0 with a transposed A is not vector-loadable)"""
    from sat_amd import _lib, kernels
    g = torch.Generator().manual_seed(M + 3 * N + K + split)
    A = torch.randn(K, M, generator=g) if ta else torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    s0 = torch.randn(N, generator=g)
    C, s = C0.to(cuda), s0.to(cuda)
    lib = _lib.load()
    if split:
        lib.sat_gemm_force_plan(64, 64, split)
    try:
        kernels.gemm(A.to(cuda).t() if ta else A.to(cuda), B.to(cuda), C, alpha=alpha, beta=1.0,
                     colsum=s)
        torch.cuda.synchronize()
    finally:
        lib.sat_gemm_force_plan(0, 0, 0)
    Al = (A.t() if ta else A).double()
    ref = alpha * (Al @ B.double()) + C0.double()
    rs = alpha * B.double().sum(0) + s0.double()
    bound = 6e-7 * (abs(alpha) * (Al.abs() @ B.double().abs()) + C0.double().abs()) + 1e-7
    assert bool(((C.double().cpu() - ref).abs() <= bound).all())
    bs = 6e-7 * (abs(alpha) * B.double().abs().sum(0) + s0.double().abs()) + 1e-7
    assert bool(((s.double().cpu() - rs).abs() <= bs).all()), float(((s.double().cpu() - rs).abs() / bs).max())


@pytest.mark.parametrize("plan", [(0, 0, 0), (64, 64, 4), (128, 64, 3), (128, 128, 2), (64, 64, 1)])
@pytest.mark.parametrize("ta", [True, False])
def test_gemm_batched_split_colsum(cuda, plan, ta):
    """a batch of weight-gradient products over one shared X (A batch stride 0: the MHA's three
    input projections) with per-batch fused column sums, split-K over the batches' slabs"""
    from sat_amd import _lib, kernels
    g = torch.Generator().manual_seed(sum(plan) + ta)
    nb, M, N, K = 3, 256, 192, 4000
    X = torch.randn(K, M, generator=g) if ta else torch.randn(M, K, generator=g)
    B = torch.randn(nb, K, N, generator=g)
    C0 = torch.randn(nb, M, N, generator=g)
    s0 = torch.randn(nb, N, generator=g)
    C, s = C0.to(cuda), s0.to(cuda)
    Xd = X.to(cuda)
    A = (Xd.t() if ta else Xd).unsqueeze(0).expand(nb, M, K)
    lib = _lib.load()
    lib.sat_gemm_force_plan(*plan)
    try:
        kernels.gemm(A, B.to(cuda), C, alpha=-0.5, beta=1.0, colsum=s)
        torch.cuda.synchronize()
    finally:
        lib.sat_gemm_force_plan(0, 0, 0)
    Al = (X.t() if ta else X).double()
    for b in range(nb):
        ref = -0.5 * (Al @ B[b].double()) + C0[b].double()
        bound = 6e-7 * (0.5 * (Al.abs() @ B[b].double().abs()) + C0[b].double().abs()) + 1e-7
        assert bool(((C[b].double().cpu() - ref).abs() <= bound).all()), b
        rs = -0.5 * B[b].double().sum(0) + s0[b].double()
        bs = 6e-7 * (0.5 * B[b].double().abs().sum(0) + s0[b].double().abs()) + 1e-7
        assert bool(((s[b].double().cpu() - rs).abs() <= bs).all()), b


@pytest.mark.parametrize("plan", [(0, 0, 0), (64, 64, 4), (128, 128, 2), (64, 64, 1)])
def test_gemm_wgrad_batch_shared_b(cuda, plan):
    """kernels.gemm_wgrad_batch: two X blocks (strided views of two buffers, equally spaced by
    construction) against one dY, the two dW blocks of one kernel, the bias column sum once
    (bias_sbatch 0: batch 0 only) -- the decoder LSTM kernels' weight gradients"""
    from sat_amd import _lib, kernels
    g = torch.Generator().manual_seed(sum(plan) + 5)
    K_, M, N = 3000, 256, 1024
    arena = torch.randn(2, K_, M + 32, generator=g).to(cuda)       # padded rows, like H2S views
    Xs = [arena[0, :, :M], arena[1, :, :M]]
    dY = torch.randn(K_, N, generator=g)
    W0 = torch.randn(2 * M, N, generator=g)
    s0 = torch.randn(N, generator=g)
    W, s = W0.to(cuda), s0.to(cuda)
    lib = _lib.load()
    lib.sat_gemm_force_plan(*plan)
    try:
        kernels.gemm_wgrad_batch(Xs, dY.to(cuda), [W[:M], W[M:]], colsum=s)
        torch.cuda.synchronize()
    finally:
        lib.sat_gemm_force_plan(0, 0, 0)
    Xh = arena.double().cpu()
    for b in range(2):
        ref = Xh[b, :, :M].t() @ dY.double() + W0[b * M:(b + 1) * M].double()
        bound = 6e-7 * ((Xh[b, :, :M].abs().t() @ dY.double().abs()) +
                        W0[b * M:(b + 1) * M].double().abs()) + 1e-7
        assert bool(((W[b * M:(b + 1) * M].double().cpu() - ref).abs() <= bound).all()), b
    rs = dY.double().sum(0) + s0.double()
    assert bool(((s.double().cpu() - rs).abs() <= 6e-7 * (dY.double().abs().sum(0) +
                                                          s0.double().abs()) + 1e-7).all())
    with pytest.raises(ValueError):
        kernels.gemm_wgrad_batch([Xs[0], Xs[1][:, :M - 4]], dY.to(cuda), [W[:M], W[M:]])


@pytest.mark.parametrize("M,K", [(256, 16000), (100, 3000), (64, 1024)])
@pytest.mark.parametrize("with_colsum", [True, False])
def test_gemm_n1_transposed_a(cuda, M, K, with_colsum):
    """N == 1 weight gradient dw = X^T dy (+ the bias sum) on gemm_tn1_kernel + the split-K
    reduce: alpha / beta / colsum against float64"""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(M + K)
    X = torch.randn(K, M, generator=g)
    dy = torch.randn(K, 1, generator=g)
    w0 = torch.randn(M, 1, generator=g)
    s0 = torch.randn(1, generator=g)
    w, s = w0.to(cuda), s0.to(cuda)
    kernels.gemm(X.to(cuda).t(), dy.to(cuda), w, alpha=-0.5, beta=1.0,
                 colsum=s if with_colsum else None)
    torch.cuda.synchronize()
    ref = -0.5 * (X.double().t() @ dy.double()) + w0.double()
    bound = 6e-7 * (0.5 * (X.double().abs().t() @ dy.double().abs()) + w0.double().abs()) + 1e-7
    assert bool(((w.double().cpu() - ref).abs() <= bound).all())
    if with_colsum:
        rs = -0.5 * dy.double().sum() + s0.double()
        assert abs(float(s.double().cpu()[0] - rs[0])) <= 6e-7 * (0.5 * float(dy.abs().sum()) +
                                                                abs(float(s0[0]))) + 1e-7


def test_gemm_colsum_fused_strided_b(cuda):
    """the attention query-layer shape: B is one tile of a [T'B, tiles, D1+D2] partial arena"""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(11)
    TB, tiles, D1, D2, A = 4000, 3, 128, 64, 128
    H = torch.randn(TB, A, generator=g)
    DQ = torch.randn(TB, tiles, D1 + D2, generator=g)
    W0, b0 = torch.randn(A, D1, generator=g), torch.randn(D1, generator=g)
    Hd, DQd, W, b = H.to(cuda), DQ.to(cuda), W0.to(cuda), b0.to(cuda)
    for t in range(tiles):
        kernels.gemm(Hd.t(), DQd[:, t, :D1], W, beta=1.0, colsum=b)
    torch.cuda.synchronize()
    ref = W0.double() + H.double().t() @ DQ[:, :, :D1].double().sum(1)
    rb = b0.double() + DQ[:, :, :D1].double().sum((0, 1))
    bound = 1e-6 * (W0.double().abs() + H.double().abs().t() @ DQ[:, :, :D1].double().abs().sum(1)) + 1e-7
    assert bool(((W.double().cpu() - ref).abs() <= bound).all())
    bb = 1e-6 * (b0.double().abs() + DQ[:, :, :D1].double().abs().sum((0, 1))) + 1e-7
    assert bool(((b.double().cpu() - rb).abs() <= bb).all())


@pytest.mark.parametrize("M", [1, 700, 25000])
def test_colsum_scatter(cuda, M):
    """sat_colsum_scatter == one column sum per destination segment (beta 1 accumulates)"""
    from sat_amd import kernels
    from sat_amd.kernels import Workspace
    g = torch.Generator().manual_seed(M)
    lens = [128, 32 * 128, 31 * 32, 32, 128]
    C = sum(lens) + 5                                    # trailing columns feed no segment
    X = torch.randn(M, C, generator=g)
    dst0 = [torch.randn(n, generator=g) for n in lens]
    dst = [d.to(cuda) for d in dst0]
    kernels.colsum_scatter(X.to(cuda), dst, Workspace(cuda), beta=1.0)
    torch.cuda.synchronize()
    cs = X.double().sum(0)
    o = 0
    for d0, d in zip(dst0, dst):
        ref = d0.double() + cs[o:o + d0.numel()]
        bound = 1e-6 * (d0.double().abs() + X[:, o:o + d0.numel()].double().abs().sum(0)) + 1e-7
        assert bool(((d.double().cpu() - ref).abs() <= bound).all())
        o += d0.numel()


@pytest.mark.parametrize("M,N,K,bm,bn,split", [(256, 1024, 3000, 64, 64, 8), (100, 36, 5000, 128, 64, 16),
                                               (130, 257, 4100, 64, 128, 4)])
def test_gemm_splitk_repeatable(cuda, M, N, K, bm, bn, split):
    """forced split-K plans: repeated launches on one stream give bit-identical results (the
    slabs are summed in a fixed order), within the fp32 bound of the float64 product"""
    from sat_amd import _lib, kernels
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A, B = torch.randn(M, K, generator=g), torch.randn(K, N, generator=g)
    Ad, Bd = A.to(cuda), B.to(cuda)
    lib = _lib.load()
    lib.sat_gemm_force_plan(bm, bn, split)
    try:
        outs = [kernels.gemm(Ad, Bd) for _ in range(4)]
        torch.cuda.synchronize()
    finally:
        lib.sat_gemm_force_plan(0, 0, 0)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    ref = A.double() @ B.double()
    bound = 6e-7 * (A.double().abs() @ B.double().abs()) + 1e-7
    assert bool(((outs[0].double().cpu() - ref).abs() <= bound).all())


@pytest.mark.parametrize("M,N,K,ta", [(16000, 1, 256, False), (37, 1, 5, False), (300, 1, 1024, True),
                                      (16000, 256, 1, False), (5, 3, 1, False), (1, 1, 1, False)])
@pytest.mark.parametrize("act", [None, "sigmoid"])
def test_gemm_degenerate_shapes(cuda, M, N, K, ta, act):
    """N == 1 (row-contiguous A: one wave per row; transposed A: the tiled path) and K == 1
    (outer product) with bias, activation and beta, against float64"""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(M + 7 * N + 3 * K)
    A = torch.randn(K, M, generator=g) if ta else torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    bias, C0 = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    C = C0.to(cuda)
    Ad = A.to(cuda).t() if ta else A.to(cuda)
    kernels.gemm(Ad, B.to(cuda), C, alpha=0.5, beta=0.75, bias=bias.to(cuda), act=act)
    torch.cuda.synchronize()
    Al = (A.t() if ta else A).double()
    ref = 0.5 * (Al @ B.double()) + 0.75 * C0.double() + bias.double()
    if act == "sigmoid":
        ref = torch.sigmoid(ref)
    bound = 2e-6 * (0.5 * (Al.abs() @ B.double().abs()) + C0.double().abs() + 1) + 1e-6
    assert bool(((C.double().cpu() - ref).abs() <= bound).all())


# ---- skinny products (M <= 8: the free-running decoder's per-step projections at batch 8)
@pytest.mark.parametrize("M,N,K", [(1, 256, 80), (3, 164, 256), (8, 768, 256), (8, 1024, 800),
                                   (5, 37, 19), (2, 50, 300), (7, 130, 33)])
@pytest.mark.parametrize("act", [None, "relu", "tanh"])
def test_gemm_skinny(cuda, M, N, K, act):
    from sat_amd import kernels
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(M, K + 3, generator=g)[:, 2:2 + K]          # strided rows (a_sm = K + 3)
    B = torch.randn(K, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g)
    add = torch.randn(M, N, generator=g)
    C = C0.to(cuda)
    kernels.gemm(A.to(cuda), B.to(cuda), C, alpha=0.5, beta=1.0, bias=bias.to(cuda), act=act,
                 add=add.to(cuda))
    torch.cuda.synchronize()
    pre = 0.5 * (A.double() @ B.double()) + C0.double() + bias.double()
    ref = {None: pre, "relu": pre.clamp_min(0), "tanh": torch.tanh(pre)}[act] + add.double()
    bound = 2e-6 * (0.5 * (A.double().abs() @ B.double().abs()) + C0.double().abs() + 1) + 1e-6
    assert bool(((C.double().cpu() - ref).abs() <= bound).all())


@pytest.mark.parametrize("M,N,K1,K2", [(16000, 1024, 256, 288), (300, 260, 64, 96),
                                       (64, 64, 2048, 4096), (96, 160, 32, 2000)])
@pytest.mark.parametrize("tb", [False, True])
def test_gemm_two_a_segments(cuda, M, N, K1, K2, tb):
    """SatGemmDesc.A2: C = [A | A2] B + bias as ONE reduction, A2 a strided column block of a
    wider buffer (as LSTM1's context input inside REC0); long K exercises split-K chunks that
    start inside the second segment."""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(M + K2)
    A = torch.randn(M, K1, generator=g)
    wide = torch.randn(M, K2 + 40, generator=g)           # A2 = wide[:, :K2] (row stride K2+40)
    B = torch.randn(N, K1 + K2, generator=g) if tb else torch.randn(K1 + K2, N, generator=g)
    bias = torch.randn(N, generator=g)
    Bd = B.to(cuda)
    wd = wide.to(cuda)
    C = kernels.gemm(A.to(cuda), Bd.t() if tb else Bd, bias=bias.to(cuda), A2=wd[:, :K2])
    Al = torch.cat([A, wide[:, :K2]], 1).double()
    Bl = (B.t() if tb else B).double()
    ref = Al @ Bl + bias.double()
    # fp32 rounding of the reduction: the 128 x 256 tile (the step's plan at 16000 x 1024 x 544)
    # accumulates each output in ONE MFMA chain over K (as a BLAS sgemm does), the smaller tiles
    # in two or four: max error 4.5e-7 vs 2.2e-7 of |A||B| over the 16 M outputs, mean 2.0e-8 vs
    # 1.5e-8 (tools/probes/seg_err.py); the deterministic bound would be K u = 3.3e-5
    bound = 8e-7 * (Al.abs() @ Bl.abs() + bias.double().abs()) + 1e-7
    err = (C.double().cpu() - ref).abs()
    assert bool((err <= bound).all()), float((err / bound).max())


@pytest.mark.parametrize("with_b2", [False, True])
def test_gemm_segments_outside_fused_path_split(cuda, with_b2):
    """Segments the fused LDS reduction cannot take (k1 = 48 is not a multiple of the 32-wide
    K-tile) run as two accumulating launches with the bias / add / beta epilogue applied once;
    a non-linear epilogue there is refused."""
    from sat_amd import _lib, kernels
    g = torch.Generator().manual_seed(48)
    A, A2 = torch.randn(64, 48, generator=g), torch.randn(64, 36, generator=g)
    B = torch.randn(48 + (0 if with_b2 else 36), 80, generator=g)
    B2 = torch.randn(36, 80, generator=g)
    C0, bias, add = torch.randn(64, 80, generator=g), torch.randn(80, generator=g), \
        torch.randn(64, 80, generator=g)
    C = C0.to(cuda)
    kernels.gemm(A.to(cuda), B.to(cuda), C, alpha=0.5, beta=-1.0, bias=bias.to(cuda),
                 add=add.to(cuda), A2=A2.to(cuda), B2=B2.to(cuda) if with_b2 else None)
    Bf = torch.cat([B, B2]) if with_b2 else B
    ref = 0.5 * (torch.cat([A, A2], 1).double() @ Bf.double()) - C0.double() + bias.double() + \
        add.double()
    bound = 4e-7 * (torch.cat([A, A2], 1).double().abs() @ Bf.double().abs() + C0.double().abs() +
                    add.double().abs() + 1)
    assert bool(((C.double().cpu() - ref).abs() <= bound).all())
    with pytest.raises(_lib.SatLibraryError):
        kernels.gemm(A.to(cuda), B.to(cuda), act="relu", A2=A2.to(cuda),
                     B2=B2.to(cuda) if with_b2 else None)


@pytest.mark.parametrize("M,N1,N2,K", [(16000, 256, 288, 1024), (300, 128, 100, 64), (70, 256, 4, 2000)])
@pytest.mark.parametrize("tb", [False, True])
def test_gemm_two_c_segments(cuda, M, N1, N2, K, tb):
    """SatGemmDesc.C2: the columns of ONE product split between two outputs (as dL/dh0' and the
    context gradients inside RD); bits equal the two separate products'."""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(M + N2)
    A = torch.randn(M, K, generator=g).to(cuda)
    B = torch.randn(N1 + N2, K, generator=g).to(cuda) if tb else \
        torch.randn(K, N1 + N2, generator=g).to(cuda)
    Bv = B.t() if tb else B
    C = torch.empty(M, N1, device=cuda)
    wide = torch.full((M, N2 + 40), 7.0, device=cuda)     # C2 = wide[:, :N2]
    kernels.gemm(A, Bv, C, C2=wide[:, :N2])
    ref = A.double().cpu() @ Bv.double().cpu()
    full = torch.cat([C, wide[:, :N2]], 1).double().cpu()
    bound = 4e-7 * (A.double().abs().cpu() @ Bv.double().abs().cpu()) + 1e-7
    assert bool(((full - ref).abs() <= bound).all())
    assert bool((wide[:, N2:] == 7.0).all())                # nothing written past C2's columns


@pytest.mark.parametrize("M,N,K1,K2", [(6400, 128, 128, 128), (300, 260, 64, 96), (64, 64, 2048, 4096)])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("with_a2", [False, True])
def test_gemm_two_b_segments(cuda, M, N, K1, K2, tb, with_a2):
    """SatGemmDesc.B2 (+ A2): C = beta C + A B + A2 B2 as ONE reduction over two separately
    stored operand pairs (as the highway layer's dx += dh W_H^T + dt W_T^T)."""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(M + K2 + 2 * tb + with_a2)
    A = torch.randn(M, K1, generator=g)
    A2 = torch.randn(M, K2, generator=g)
    Bs = [torch.randn(N, k, generator=g) if tb else torch.randn(k, N, generator=g) for k in (K1, K2)]
    C0 = torch.randn(M, N, generator=g)
    Bd = [b.to(cuda) for b in Bs]
    Bv = [b.t() if tb else b for b in Bd]
    C = C0.to(cuda)
    if with_a2:
        kernels.gemm(A.to(cuda), Bv[0], C, beta=1.0, A2=A2.to(cuda), B2=Bv[1])
    else:
        kernels.gemm(torch.cat([A, A2], 1).to(cuda), Bv[0], C, beta=1.0, B2=Bv[1])
    Bl = [(b.t() if tb else b).double() for b in Bs]
    ref = C0.double() + A.double() @ Bl[0] + A2.double() @ Bl[1]
    bound = 4e-7 * (C0.double().abs() + A.double().abs() @ Bl[0].abs() +
                    A2.double().abs() @ Bl[1].abs()) + 1e-7
    assert bool(((C.double().cpu() - ref).abs() <= bound).all())


def test_gemm_two_segments_batched(cuda):
    """A2 / B2 on a batched product (the encoder BiLSTM's input gradient: per position n,
    dhw[:, n] = DG_fw[n] Wx_fw^T + DG_bw[n] Wx_bw^T, written transposed)."""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(11)
    N, B, G4, Win = 37, 6, 512, 128
    DG = [torch.randn(N, B, G4, generator=g) for _ in range(2)]
    W = [torch.randn(Win + 64, G4, generator=g) for _ in range(2)]   # [Win + U, 4U] kernels
    out = torch.full((B, N, Win), float("nan"), device=cuda)
    Wd = [w.to(cuda) for w in W]
    kernels.gemm(DG[0].to(cuda), Wd[0][:Win].t(), out.transpose(0, 1), A2=DG[1].to(cuda),
                 B2=Wd[1][:Win].t())
    ref = sum((DG[i].double() @ W[i][:Win].double().t()).transpose(0, 1) for i in range(2))
    bound = 4e-7 * sum((DG[i].double().abs() @ W[i][:Win].double().abs().t()).transpose(0, 1)
                       for i in range(2)) + 1e-7
    assert bool(((out.double().cpu() - ref).abs() <= bound).all())


def test_gemm_batched_b2(cuda):
    """A batched B2 ([batch, K2, N]): the inner dimension is B2's second-to-last (not its batch
    count); C[i] = A[i][:, :k1] B[i] + A[i][:, k1:] B2[i]."""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(12)
    nb, M, N, K1, K2 = 3, 70, 96, 64, 32
    A = torch.randn(nb, M, K1 + K2, generator=g)
    # the second segment takes B's batch strides (SatGemmDesc has one b_sbatch): B2 is the
    # leading K2 rows of a device buffer laid out like B
    B, B2buf = torch.randn(nb, K1, N, generator=g), torch.randn(nb, K1, N, generator=g)
    B2 = B2buf[:, :K2]
    C = kernels.gemm(A.to(cuda), B.to(cuda), B2=B2buf.to(cuda)[:, :K2])
    ref = A.double() @ torch.cat([B, B2], 1).double()
    bound = 4e-7 * (A.double().abs() @ torch.cat([B, B2], 1).double().abs()) + 1e-7
    assert bool(((C.double().cpu() - ref).abs() <= bound).all())


# ---- causal structure hint (SatGemmDesc.tri): the decoder head's score / probability products
@pytest.mark.parametrize("L,K", [(200, 128), (500, 128), (77, 40)])
def test_gemm_tri(cuda, L, K):
    """tri=1 writes every entry on / below the diagonal (above it C is left as it was); tri=2 / 3
    with a lower / upper triangular A give the same bits as the full product."""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(L + K)
    nb = 3
    A = torch.randn(nb, L, K, generator=g).to(cuda)
    Bm = torch.randn(nb, K, L, generator=g).to(cuda)
    C = torch.full((nb, L, L), float("nan"), device=cuda)
    kernels.gemm(A, Bm, C, tri=1)
    ref = kernels.gemm(A, Bm)
    low = torch.ones(L, L, device=cuda).tril().bool()
    assert bool((C[:, low] == ref[:, low]).all())
    P = torch.randn(nb, L, L, generator=g).to(cuda)
    V = torch.randn(nb, L, K, generator=g).to(cuda)
    for tri, Pt in ((2, P.tril()), (3, P.triu())):
        full = kernels.gemm(Pt, V)
        part = kernels.gemm(Pt, V, tri=tri)
        assert torch.equal(full, part), tri
        # the transposed view (A_M layout) as the backward uses it: Pd^T dO / dS^T Q
        Pl = P.tril()
        full_t = kernels.gemm(Pl.transpose(1, 2), V)
        part_t = kernels.gemm(Pl.transpose(1, 2), V, tri=3)
        assert torch.equal(full_t, part_t)
    ref64 = P.tril().double() @ V.double()
    assert float((kernels.gemm(P.tril(), V, tri=2).double() - ref64).abs().max()) < 1e-3


def test_gemm_tri_batch1_long_k_never_splits(cuda):
    """a batch-1 tri=1 product with K >= 512 (a split-K shape) must still leave the
    tiles above the diagonal unwritten -- the planner takes no split under the hint -- and tri
    with the fused bias-gradient row or segmented operands is refused."""
    from sat_amd import _lib, kernels
    g = torch.Generator().manual_seed(9)
    L, K = 256, 1024
    A = torch.randn(L, K, generator=g).to(cuda)
    Bm = torch.randn(K, L, generator=g).to(cuda)
    C = torch.full((L, L), float("nan"), device=cuda)
    kernels.gemm(A, Bm, C, tri=1)
    ref = A.double() @ Bm.double()          # (the untriangular product may split K: other bits)
    low = torch.ones(L, L, device=cuda).tril().bool()
    err = (C.double() - ref)[low].abs() / (A.abs().double() @ Bm.abs().double())[low]
    assert float(err.max()) < 1e-6
    assert bool(torch.isnan(C[:64, 128:]).all())            # wholly above the diagonal
    with pytest.raises(_lib.SatLibraryError, match="tri cannot be combined"):
        kernels.gemm(A, Bm, torch.empty(L, L, device=cuda), tri=1,
                     colsum=torch.zeros(L, device=cuda))
    with pytest.raises(_lib.SatLibraryError, match="tri cannot be combined"):
        kernels.gemm(A[:, :512], Bm, torch.empty(L, L, device=cuda), tri=1, A2=A[:, 512:])
