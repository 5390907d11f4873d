"""sat_mha_fwd / sat_mha_bwd (the C-ABI MultiHeadAttention, modules/self_attention.py:108-128)
against the float64 oracle restatement and its autograd."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double().cpu() - b.double()).abs().max() / (b.double().abs().max() + 1e-12))


@pytest.mark.parametrize("B,L,W,D,H,out,causal,drop,flash", [
    (3, 17, 64, 64, 2, 64, True, False, False), (2, 40, 48, 64, 4, 80, False, True, False),
    (4, 200, 256, 256, 4, 256, False, True, False), (2, 250, 256, 256, 4, 256, True, True, False),
    # the decoder head's shape through the fused causal attention (dh = 128, lse kept)
    (2, 500, 256, 256, 2, 256, True, True, True), (3, 100, 64, 256, 2, 64, True, False, True),
    (2, 36, 128, 128, 1, 96, True, True, True),
    # narrow heads through the fused attention (the encoder's 2 x 16 at L = N <= 256, any mask)
    (3, 17, 64, 32, 2, 32, False, True, True), (2, 200, 256, 32, 2, 32, False, True, True),
    (2, 248, 64, 64, 2, 64, True, True, True), (1, 33, 16, 16, 2, 16, False, False, True),
    (2, 65, 48, 64, 4, 48, True, False, True)])
def test_mha_fwd_bwd_match_oracle(cuda, B, L, W, D, H, out, causal, drop, flash):
    from oracle import sat_oracle as O
    from sat_amd import kernels
    g = torch.Generator().manual_seed(B * 1000 + L)
    sc = "mha"
    p64 = {}
    for n, (i, o) in {"query": (W, D), "key": (W, D), "value": (W, D), "output": (D, out)}.items():
        p64[f"{sc}/{n}_projection/kernel"] = (torch.randn(i, o, generator=g, dtype=torch.float64)
                                              / i ** 0.5).requires_grad_(True)
        p64[f"{sc}/{n}_projection/bias"] = (0.1 * torch.randn(o, generator=g, dtype=torch.float64)
                                            ).requires_grad_(True)
    x64 = torch.randn(B, L, W, generator=g, dtype=torch.float64, requires_grad=True)
    mask = None
    if drop:
        keep = (torch.rand(B, H, L, L, generator=g) < 0.9).double() / 0.9
        mask = keep
    y64, _ = O.mha(x64, p64, sc, H, causal, mask)
    dy = torch.randn(B, L, out, generator=g, dtype=torch.float64)
    y64.backward(dy)

    P = {k: v.detach().float().to(cuda) for k, v in p64.items()}
    G = {k: torch.zeros_like(v) for k, v in P.items()}
    x = x64.detach().float().to(cuda)
    md = None if mask is None else mask.float().to(cuda)
    s = dict(x=x, q=torch.empty(B, L, D, device=cuda), k=torch.empty(B, L, D, device=cuda),
             v=torch.empty(B, L, D, device=cuda),
             o=torch.empty(B, L, D, device=cuda), y=torch.empty(B, L, out, device=cuda))
    if flash:
        s["lse"] = torch.empty(B, H, L, device=cuda)       # P / Pd never materialised
    else:
        s["P"] = torch.empty(B, H, L, L, device=cuda)
        s["Pd"] = torch.empty_like(s["P"]) if md is not None else s["P"]
    names = [f"{sc}/{n}_projection/{t}" for n in ("query", "key", "value", "output")
             for t in ("kernel", "bias")]
    d, scratch = kernels.mha_desc(x, *(P[n] for n in names), H, causal, md, s)
    kernels.mha_fwd(d)
    assert _rel(s["y"], y64.detach()) < 2e-5
    dyd = dy.float().to(cuda)
    dx = torch.empty_like(x)
    d.dy, d.dx = dyd.data_ptr(), dx.data_ptr()
    d.dWq, d.dbq, d.dWk, d.dbk, d.dWv, d.dbv, d.dWo, d.dbo = (G[n].data_ptr() for n in names)
    kernels.mha_bwd(d)
    torch.cuda.synchronize()
    assert _rel(dx, x64.grad) < 2e-5
    # the key-projection bias gradient is exactly 0 (a per-row constant in the scores cancels in
    # the softmax): every gradient is checked against the largest gradient's magnitude
    scale = max(float(p64[n].grad.abs().max()) for n in names)
    for n in names:
        err = float((G[n].double().cpu() - p64[n].grad).abs().max())
        assert err <= 2e-5 * max(scale, 1e-12), (n, err, scale)


def _attn64(q, k, v, H, mask, causal=True):
    """float64 attention per (utterance, head) on [B, L, H*dh] (self_attention.py:45-65)."""
    B, L, D = q.shape
    dh = D // H
    sp = lambda t: t.view(B, L, H, dh).transpose(1, 2)                  # noqa: E731
    s = sp(q) @ sp(k).transpose(-1, -2) / dh ** 0.5
    if causal:
        s = s.masked_fill(torch.ones(L, L, dtype=torch.bool).triu(1), float("-inf"))
    p = torch.softmax(s, -1)
    if mask is not None:
        p = p * mask
    return (p @ sp(v)).transpose(1, 2).reshape(B, L, D)


@pytest.mark.parametrize("B,H,L,drop", [(2, 2, 500, True), (1, 3, 68, False), (2, 1, 4, True),
                                        (1, 2, 132, True)])
def test_flash_attn_kernels_match_fp64(cuda, B, H, L, drop):
    """sat_flash_attn_fwd / _bwd directly (ragged last row block, one-row-block and tiny L,
    dropout mask) against float64 autograd: O, dQ, dK, dV within 2e-6 of their max."""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(L + 7 * H)
    D = 128 * H
    q64, k64, v64 = (torch.randn(B, L, D, generator=g, dtype=torch.float64, requires_grad=True)
                     for _ in range(3))
    mask = ((torch.rand(B, H, L, L, generator=g) < 0.95).double() / 0.95) if drop else None
    o64 = _attn64(q64, k64, v64, H, mask)
    do = torch.randn(B, L, D, generator=g, dtype=torch.float64)
    o64.backward(do)
    q, k, v = (t.detach().float().to(cuda) for t in (q64, k64, v64))
    md = None if mask is None else mask.float().to(cuda)
    o = torch.full((B, L, D), float("nan"), device=cuda)
    lse = torch.empty(B, H, L, device=cuda)
    kernels.flash_attn(q, k, v, o, lse, H, mask=md)
    dq, dk, dv = (torch.full((B, L, D), float("nan"), device=cuda) for _ in range(3))
    kernels.flash_attn(q, k, v, o, lse, H, mask=md, dout=do.float().to(cuda), dq=dq, dk=dk, dv=dv,
                       delta=torch.empty(B, H, L, device=cuda))
    torch.cuda.synchronize()
    for got, ref in ((o, o64.detach()), (dq, q64.grad), (dk, k64.grad), (dv, v64.grad)):
        assert _rel(got, ref) < 5e-6


def test_flash_attn_equals_materialised_path_closely(cuda, monkeypatch):
    """The decoder head at C2 size (B=32, T'=500, 2 heads of 128): the fused path against the
    materialised scores + softmax + GEMMs (SAT_FLASH_ATTN=0 route) -- same math, other
    summation order: y and every gradient within 1e-5 of their max."""
    from sat_amd import kernels
    B, L, W, D, H, out = 32, 500, 256, 256, 2, 256
    g = torch.Generator().manual_seed(5)
    P = {}
    names = []
    for nm, (i, o) in {"query": (W, D), "key": (W, D), "value": (W, D), "output": (D, out)}.items():
        P[f"m/{nm}_projection/kernel"] = (torch.randn(i, o, generator=g) / i ** 0.5).to(cuda)
        P[f"m/{nm}_projection/bias"] = (0.1 * torch.randn(o, generator=g)).to(cuda)
        names += [f"m/{nm}_projection/kernel", f"m/{nm}_projection/bias"]
    x = torch.randn(B, L, W, generator=g).to(cuda)
    md = ((torch.rand(B, H, L, L, generator=g) < 0.95).float() / 0.95).to(cuda)
    dy = torch.randn(B, L, out, generator=g).to(cuda)
    res = []
    for flash in (True, False):
        s = dict(x=x, q=torch.empty(B, L, D, device=cuda), k=torch.empty(B, L, D, device=cuda),
                 v=torch.empty(B, L, D, device=cuda), o=torch.empty(B, L, D, device=cuda),
                 y=torch.empty(B, L, out, device=cuda))
        if flash:
            s["lse"] = torch.empty(B, H, L, device=cuda)
        else:
            s["P"] = torch.empty(B, H, L, L, device=cuda)
            s["Pd"] = torch.empty_like(s["P"])
        G = {n: torch.zeros_like(P[n]) for n in names}
        d, scratch = kernels.mha_desc(x, *(P[n] for n in names), H, True, md, s)
        kernels.mha_fwd(d)
        dx = torch.empty_like(x)
        d.dy, d.dx = dy.data_ptr(), dx.data_ptr()
        d.dWq, d.dbq, d.dWk, d.dbk, d.dWv, d.dbv, d.dWo, d.dbo = (G[n].data_ptr() for n in names)
        kernels.mha_bwd(d)
        torch.cuda.synchronize()
        res.append((s["y"].clone(), dx, G))
    (y1, dx1, G1), (y2, dx2, G2) = res
    assert _rel(y1, y2.cpu()) < 1e-5
    assert _rel(dx1, dx2.cpu()) < 1e-5
    # (the key-projection bias gradient is exactly 0 in exact arithmetic -- rounding noise on
    # both sides -- so every gradient is held to the largest gradient's magnitude)
    gmax = max(float(G2[n].abs().max()) for n in names)
    for n in names:
        assert float((G1[n] - G2[n]).abs().max()) <= 1e-5 * gmax, n


@pytest.mark.parametrize("B,H,L,dh,causal,drop", [
    (2, 2, 200, 16, False, True), (3, 2, 17, 16, False, True), (1, 3, 256, 16, True, True),
    (2, 1, 1, 16, False, False), (2, 2, 130, 32, False, True), (1, 2, 248, 32, True, False),
    (2, 4, 64, 8, False, True), (1, 1, 5, 8, True, True)])
def test_narrow_flash_attn_kernels_match_fp64(cuda, B, H, L, dh, causal, drop):
    """sat_flash_attn_fwd / _bwd on narrow heads (the encoder's self-attention shape: dh <= 32,
    L <= 256; ragged last row block, one-row and full-LDS cases, causal or not, dropout mask)
    against float64 autograd: O, dQ, dK, dV within 5e-6 of their max."""
    from sat_amd import kernels
    g = torch.Generator().manual_seed(L + 7 * H + dh)
    D = dh * H
    q64, k64, v64 = (torch.randn(B, L, D, generator=g, dtype=torch.float64, requires_grad=True)
                     for _ in range(3))
    mask = ((torch.rand(B, H, L, L, generator=g) < 0.9).double() / 0.9) if drop else None
    o64 = _attn64(q64, k64, v64, H, mask, causal)
    do = torch.randn(B, L, D, generator=g, dtype=torch.float64)
    o64.backward(do)
    q, k, v = (t.detach().float().to(cuda) for t in (q64, k64, v64))
    md = None if mask is None else mask.float().to(cuda)
    o = torch.full((B, L, D), float("nan"), device=cuda)
    lse = torch.empty(B, H, L, device=cuda)
    kernels.flash_attn(q, k, v, o, lse, H, mask=md, causal=causal)
    dq, dk, dv = (torch.full((B, L, D), float("nan"), device=cuda) for _ in range(3))
    kernels.flash_attn(q, k, v, o, lse, H, mask=md, dout=do.float().to(cuda), dq=dq, dk=dk, dv=dv,
                       causal=causal)
    torch.cuda.synchronize()
    for got, ref in ((o, o64.detach()), (dq, q64.grad), (dk, k64.grad), (dv, v64.grad)):
        assert _rel(got, ref) < 5e-6


def test_narrow_flash_refuses_what_it_cannot_hold(cuda):
    """L > 256, dh outside {8, 16, 32} (other than the causal 128) and more LDS than 64 KB are
    refused with the library's argument error, never run."""
    from sat_amd import _lib, kernels
    for B, H, L, dh, causal in ((1, 2, 257, 16, False), (1, 2, 64, 24, False),
                                (1, 1, 256, 32, False), (1, 1, 64, 128, False)):
        q = torch.zeros(B, L, H * dh, device=cuda)
        with pytest.raises(_lib.SatLibraryError):
            kernels.flash_attn(q, q, q, torch.empty_like(q), torch.empty(B, H, L, device=cuda), H,
                               causal=causal)


def test_narrow_flash_equals_materialised_path_closely(cuda):
    """The encoder's self-attention at C2 size (B=32, N=200, 2 heads of 16, dropout): the fused
    path against the materialised scores + softmax + GEMMs -- y and every gradient within 1e-5 of
    their max."""
    from sat_amd import kernels
    B, L, W, D, H, out = 32, 200, 256, 32, 2, 32
    g = torch.Generator().manual_seed(11)
    P = {}
    names = []
    for nm, (i, o) in {"query": (W, D), "key": (W, D), "value": (W, D), "output": (D, out)}.items():
        P[f"m/{nm}_projection/kernel"] = (torch.randn(i, o, generator=g) / i ** 0.5).to(cuda)
        P[f"m/{nm}_projection/bias"] = (0.1 * torch.randn(o, generator=g)).to(cuda)
        names += [f"m/{nm}_projection/kernel", f"m/{nm}_projection/bias"]
    x = torch.randn(B, L, W, generator=g).to(cuda)
    md = ((torch.rand(B, H, L, L, generator=g) < 0.9).float() / 0.9).to(cuda)
    dy = torch.randn(B, L, out, generator=g).to(cuda)
    res = []
    for flash in (True, False):
        s = dict(x=x, q=torch.empty(B, L, D, device=cuda), k=torch.empty(B, L, D, device=cuda),
                 v=torch.empty(B, L, D, device=cuda), o=torch.empty(B, L, D, device=cuda),
                 y=torch.empty(B, L, out, device=cuda))
        if flash:
            s["lse"] = torch.empty(B, H, L, device=cuda)
        else:
            s["P"] = torch.empty(B, H, L, L, device=cuda)
            s["Pd"] = torch.empty_like(s["P"])
        G = {n: torch.zeros_like(P[n]) for n in names}
        d, scratch = kernels.mha_desc(x, *(P[n] for n in names), H, False, md, s)
        kernels.mha_fwd(d)
        dx = torch.empty_like(x)
        d.dy, d.dx = dy.data_ptr(), dx.data_ptr()
        d.dWq, d.dbq, d.dWk, d.dbk, d.dWv, d.dbv, d.dWo, d.dbo = (G[n].data_ptr() for n in names)
        kernels.mha_bwd(d)
        torch.cuda.synchronize()
        res.append((s["y"].clone(), dx, G))
    (y1, dx1, G1), (y2, dx2, G2) = res
    assert _rel(y1, y2.cpu()) < 1e-5
    assert _rel(dx1, dx2.cpu()) < 1e-5
    gmax = max(float(G2[n].abs().max()) for n in names)
    for n in names:
        assert float((G1[n] - G2[n]).abs().max()) <= 1e-5 * gmax, n


@pytest.mark.parametrize("flash", [True, False])
def test_deferred_weight_gradients_equal_inline(cuda, flash):
    """sat_mha_bwd with the four weight gradients NULL (dx only) followed by sat_mha_bwd_wgrad on
    the same scratch gives bitwise the inline call's dx and parameter gradients (the decoder
    head's shape through the fused attention, and the materialised path)."""
    from sat_amd import kernels
    B, L, W, D, H, out = 2, 96, 64, 256, 2, 64
    g = torch.Generator().manual_seed(21)
    P, names = {}, []
    for nm, (i, o) in {"query": (W, D), "key": (W, D), "value": (W, D), "output": (D, out)}.items():
        P[f"m/{nm}_projection/kernel"] = (torch.randn(i, o, generator=g) / i ** 0.5).to(cuda)
        P[f"m/{nm}_projection/bias"] = (0.1 * torch.randn(o, generator=g)).to(cuda)
        names += [f"m/{nm}_projection/kernel", f"m/{nm}_projection/bias"]
    x = torch.randn(B, L, W, generator=g).to(cuda)
    md = ((torch.rand(B, H, L, L, generator=g) < 0.9).float() / 0.9).to(cuda)
    dy = torch.randn(B, L, out, generator=g).to(cuda)
    res = []
    for deferred in (False, True):
        s = dict(x=x, q=torch.empty(B, L, D, device=cuda), k=torch.empty(B, L, D, device=cuda),
                 v=torch.empty(B, L, D, device=cuda), o=torch.empty(B, L, D, device=cuda),
                 y=torch.empty(B, L, out, device=cuda))
        if flash:
            s["lse"] = torch.empty(B, H, L, device=cuda)
        else:
            s["P"] = torch.empty(B, H, L, L, device=cuda)
            s["Pd"] = torch.empty_like(s["P"])
        G = {n: torch.zeros_like(P[n]) for n in names}
        d, scratch = kernels.mha_desc(x, *(P[n] for n in names), H, True, md, s)
        kernels.mha_fwd(d)
        dx = torch.empty_like(x)
        d.dy, d.dx = dy.data_ptr(), dx.data_ptr()
        grads = [G[n].data_ptr() for n in names]
        if deferred:
            kernels.mha_bwd(d)
            d.dWq, d.dbq, d.dWk, d.dbk, d.dWv, d.dbv, d.dWo, d.dbo = grads
            kernels.mha_bwd_wgrad(d)
        else:
            d.dWq, d.dbq, d.dWk, d.dbk, d.dWv, d.dbv, d.dWo, d.dbo = grads
            kernels.mha_bwd(d)
        torch.cuda.synchronize()
        res.append((dx, G))
    (dx1, G1), (dx2, G2) = res
    assert torch.equal(dx1, dx2)
    for n in names:
        assert torch.equal(G1[n], G2[n]), n
