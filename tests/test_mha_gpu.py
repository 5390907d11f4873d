"""sat_mha_fwd / sat_mha_bwd (the C-ABI MultiHeadAttention, modules/self_attention.py:108-128)
against the float64 oracle restatement and its autograd."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double().cpu() - b.double()).abs().max() / (b.double().abs().max() + 1e-12))


@pytest.mark.parametrize("B,L,W,D,H,out,causal,drop", [
    (3, 17, 64, 64, 2, 64, True, False), (2, 40, 48, 64, 4, 80, False, True),
    (4, 200, 256, 256, 4, 256, False, True), (2, 250, 256, 256, 4, 256, True, True)])
def test_mha_fwd_bwd_match_oracle(cuda, B, L, W, D, H, out, causal, drop):
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
             v=torch.empty(B, L, D, device=cuda), P=torch.empty(B, H, L, L, device=cuda),
             o=torch.empty(B, L, D, device=cuda), y=torch.empty(B, L, out, device=cuda))
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
