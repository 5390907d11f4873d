"""Memory-bound step kernels against CPU references: the self-attention row softmax
(sat_softmax_fwd/bwd; register-resident rows up to 1024 columns, streaming beyond; torch fp64),
the CBHG max pooling (sat_maxpool2/_bwd; exact, ties included) and the embedding gradient
(sat_embedding_bwd; exact row-ordered float32 sums)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("L", [7, 200, 256, 500, 1000, 1500])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("dropout", [False, True])
def test_softmax_fwd_bwd(cuda, L, causal, dropout):
    from sat_amd import kernels as K
    g = torch.Generator().manual_seed(L + 2 * causal + dropout)
    Bh, Lq = 6, L                        # [B*H, Lq, L] score rows (causal: square)
    scale = 0.125
    S = torch.randn(Bh, Lq, L, generator=g) * 4
    mask = (torch.rand(Bh, Lq, L, generator=g) > 0.1).float() / 0.9 if dropout else None
    dPd = torch.randn(Bh, Lq, L, generator=g)
    Sd = S.to(cuda)
    P = torch.empty_like(Sd)
    Pd = torch.empty_like(Sd) if dropout else None
    md = mask.to(cuda) if dropout else None
    K.softmax_fwd(Sd, P, Pd, mask=md, causal=causal, scale=scale)
    dS = torch.empty_like(Sd)
    dPg = dPd.to(cuda)
    if causal:    # above the diagonal dPd is never read (the score GEMM leaves it unwritten)
        dPg.masked_fill_(torch.ones(Lq, L, device=cuda).triu(1).bool(), float("nan"))
    K.softmax_bwd(P, dPg, dS, mask=md, scale=scale, causal=causal)
    torch.cuda.synchronize()

    x = S.double() * scale
    if causal:
        x = x.masked_fill(torch.ones(Lq, L).triu(1).bool(), float("-inf"))
    ref = torch.softmax(x, -1)
    assert float((P.double().cpu() - ref).abs().max()) < 2e-6
    if dropout:
        assert float((Pd.double().cpu() - ref * mask.double()).abs().max()) < 2e-5
    dp = dPd.double() * (mask.double() if dropout else 1.0)
    dref = scale * ref * (dp - (dp * ref).sum(-1, keepdim=True))
    assert float((dS.double().cpu() - dref).abs().max()) < 5e-6 * (1 + float(dp.abs().max()))
    if causal:                          # masked columns are exact zeros
        up = torch.ones(Lq, L).triu(1).bool().expand(Bh, Lq, L)
        assert float(P.cpu()[up].abs().max()) == 0.0 if up.any() else True


def _maxpool_ref(x, dy):
    """MaxPooling1D(2, stride 1, SAME) and its gradient, first index winning ties"""
    nxt = torch.cat([x[:, 1:], x[:, -1:]], 1)
    last = torch.zeros_like(x, dtype=torch.bool)
    last[:, -1] = True
    y = torch.where(last, x, torch.maximum(x, nxt))
    own = last | (x >= nxt)
    dx = torch.where(own, dy, torch.zeros_like(dy))
    prv = torch.cat([x[:, :1], x[:, :-1]], 1)
    dprv = torch.cat([torch.zeros_like(dy[:, :1]), dy[:, :-1]], 1)
    first = torch.zeros_like(x, dtype=torch.bool)
    first[:, 0] = True
    dx = dx + torch.where(~first & (prv < x), dprv, torch.zeros_like(dy))
    return y, dx


@pytest.mark.parametrize("B,N,C", [(3, 17, 2048), (2, 1, 128), (4, 9, 7), (32, 200, 128),
                                   (32, 200, 2048), (16, 203, 2048), (64, 9, 1024)])
def test_maxpool2_fwd_bwd(cuda, B, N, C):
    """float4 paths (C % 4 == 0; chunked backward at >= 65536 threads, ragged last chunk
    included) and the scalar path, with ties (quantised inputs)"""
    from sat_amd import kernels as K
    g = torch.Generator().manual_seed(B * N + C)
    x = torch.randint(-3, 4, (B, N, C), generator=g).float()
    dy = torch.randn(B, N, C, generator=g)
    xd = x.to(cuda)
    y = K.maxpool2(xd, torch.empty_like(xd))
    dx = K.maxpool2_bwd(xd, dy.to(cuda), torch.empty_like(xd))
    torch.cuda.synchronize()
    yr, dxr = _maxpool_ref(x, dy)
    assert torch.equal(y.cpu(), yr)
    assert torch.equal(dx.cpu(), dxr)


@pytest.mark.parametrize("B,N,C", [(32, 200, 2048), (3, 17, 2048), (2, 1, 128), (4, 9, 7),
                                   (16, 203, 256)])
@pytest.mark.parametrize("relu", [True, False])
def test_bn_apply_maxpool2_fused(cuda, B, N, C, relu):
    """sat_bn_apply_maxpool2 (the conv bank's BN + max-pool in one pass, ragged last chunk and
    the two-launch fallback at C % 4 != 0) == sat_bn_apply then sat_maxpool2, bitwise"""
    from sat_amd import kernels as K
    g = torch.Generator().manual_seed(B * N + C + relu)
    x = (torch.randn(B, N, C, generator=g) * 2).to(cuda)
    mean = torch.randn(C, generator=g).to(cuda)
    var = torch.rand(C, generator=g).to(cuda) + 0.1
    gam = torch.randn(C, generator=g).to(cuda)
    bet = torch.randn(C, generator=g).to(cuda)
    y1 = torch.empty_like(x)
    K.bn_apply(x.view(-1, C), y1.view(-1, C), mean, var, gam, bet, relu=relu)
    mp1 = K.maxpool2(y1, torch.empty_like(x))
    y2, mp2 = torch.empty_like(x), torch.empty_like(x)
    K.bn_apply_maxpool2(x, y2, mp2, mean, var, gam, bet, relu=relu)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert torch.equal(mp1, mp2)


@pytest.mark.parametrize("R,D,V,offset", [(6400, 512, 70, 0), (37, 300, 5, 3), (1, 512, 4, 0),
                                          (1100, 64, 1, 0), (8192, 256, 9, 0), (9000, 64, 3, 0)])
def test_embedding_bwd_row_order(cuda, R, D, V, offset):
    """dtable[v] += sum of the dout rows whose id hits v, added in row order (bit-exact against
    the same float32 sequence on the CPU); rows never hit stay untouched"""
    from sat_amd import kernels as K
    g = torch.Generator().manual_seed(R + D + V)
    ids = torch.randint(offset, offset + V, (R,), generator=g)
    if V > 2:
        ids[ids == offset + 1] = offset     # one table row never hit
    dout = torch.randn(R, D, generator=g)
    table0 = torch.randn(V, D, generator=g)
    dt = table0.to(cuda)
    K.embedding_bwd(dout.to(cuda), ids.to(cuda), dt, offset=offset)
    torch.cuda.synchronize()
    ref = table0.clone()
    for v in range(V):
        rows = (ids - offset == v).nonzero().flatten().tolist()
        if not rows:
            continue
        acc = torch.zeros(D)
        for r in rows:
            acc = acc + dout[r]
        ref[v] = ref[v] + acc
    assert torch.equal(dt.cpu(), ref)


@pytest.mark.parametrize("B,T,M,Tp", [(32, 1000, 80, 500), (3, 17, 7, 9), (2, 8, 4, 4)])
def test_loss_partials(cuda, B, T, M, Tp):
    """sat_loss_fwd_bwd's values against float64 CPU: masked L1 over the mel rows (rows of weight 0
    skipped even when they hold NaN), masked BCE of the stop logits, their counts"""
    from sat_amd import kernels as K
    g = torch.Generator().manual_seed(B * T + M)
    mel, tgt = torch.randn(B, T, M, generator=g), torch.randn(B, T, M, generator=g)
    tmask = (torch.rand(B, T, generator=g) > 0.3).float()
    mel[tmask == 0] = float("nan")
    stop, done = torch.randn(B, Tp, generator=g), (torch.rand(B, Tp, generator=g) > 0.5).float()
    dmask = (torch.rand(B, Tp, generator=g) > 0.2).float()
    out = torch.zeros(8, device=cuda)
    K.loss_fwd_bwd(mel.to(cuda), tgt.to(cuda), tmask.to(cuda), stop.to(cuda), done.to(cuda),
                   dmask.to(cuda), out)
    torch.cuda.synchronize()
    w = tmask.double()[..., None]
    d = torch.where(w > 0, (mel.double() - tgt.double()).abs(), torch.zeros(()).double())
    c1 = max(float(tmask.sum()) * M, 1.0)
    L1 = float((w * d).sum()) / c1
    x, z, wd = stop.double(), done.double(), dmask.double()
    xe = x.clamp(min=0) - x * z + torch.log1p(torch.exp(-x.abs()))
    cb = max(float((dmask != 0).sum()), 1.0)
    BCE = float((wd * xe).sum()) / cb
    o = out.cpu().double()
    assert abs(float(o[1]) - L1) <= 1e-6 * abs(L1) + 1e-7
    assert abs(float(o[2]) - BCE) <= 1e-6 * abs(BCE) + 1e-7
    assert float(o[3]) == c1 and float(o[4]) == cb
    assert abs(float(o[0]) - (0.1 * L1 + BCE)) <= 1e-6 * (0.1 * L1 + BCE) + 1e-7


@pytest.mark.parametrize("M,C,strided", [(6400, 128, False), (6400, 2048, False), (37, 6, False),
                                         (300, 64, True)])
def test_batchnorm_passes(cuda, M, C, strided):
    """sat_bn_stats / sat_bn_apply (ReLU, residual) / sat_bn_bwd (ReLU gate, beta_out) against
    float64 CPU; float4 paths (C % 4 == 0) and scalar path, row-strided views included"""
    from sat_amd import kernels as K
    g = torch.Generator().manual_seed(M + C)
    eps = 1e-3
    xb = torch.randn(M, 2 * C if strided else C, generator=g) * 2 + 0.5
    x = xb[:, :C]
    gamma, beta = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)
    res, dy = torch.randn(M, C, generator=g), torch.randn(M, C, generator=g)
    dx0 = torch.randn(M, C, generator=g)
    ws = K.Workspace(cuda)
    xd = xb.to(cuda)[:, :C]
    mean, var = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    K.bn_stats(xd, mean, var, ws)
    y = torch.empty(M, C, device=cuda)
    gd, bd = gamma.to(cuda), beta.to(cuda)
    K.bn_apply(xd, y, mean, var, gd, bd, relu=True, res=res.to(cuda), eps=eps)
    # backward through the ReLU: gate = post-BN ReLU output (before the residual)
    gate = (y - res.to(cuda))
    dgam, dbet = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
    dx = dx0.to(cuda)
    K.bn_bwd(dy.to(cuda), xd, gate, dx, mean, var, gd, dgam, dbet, ws, training=True,
             beta_out=1.0, eps=eps)
    torch.cuda.synchronize()

    xx = x.double()
    mu, vr = xx.mean(0), xx.var(0, unbiased=False)
    assert float((mean.cpu().double() - mu).abs().max()) < 1e-5
    assert float((var.cpu().double() - vr).abs().max()) < 1e-5 * float(vr.max())
    xh = (xx - mu) / torch.sqrt(vr + eps)
    pre = gamma.double() * xh + beta.double()
    yr = pre.clamp(min=0) + res.double()
    assert float((y.cpu().double() - yr).abs().max()) < 2e-5
    # the gate as the kernel saw it (y - res can round a tiny positive pre-activation to 0)
    gg = torch.where(gate.cpu() > 0, dy.double(), torch.zeros(()).double())
    dxr = gamma.double() / torch.sqrt(vr + eps) * (gg - gg.mean(0) - xh * (gg * xh).mean(0))
    assert float((dx.cpu().double() - (dx0.double() + dxr)).abs().max()) < 5e-5
    assert float((dbet.cpu().double() - gg.sum(0)).abs().max()) < 1e-3
    assert float((dgam.cpu().double() - (gg * xh).sum(0)).abs().max()) < 1e-3
