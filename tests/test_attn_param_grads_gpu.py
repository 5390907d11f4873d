"""sat_attn_param_grads (the attention parameter gradients summed over every decoder step,
modules/forward_attention.py:16-23, 68-122 and TF BahdanauAttention's memory / score variables)
against a torch fp64 restatement (energies recomputed from K, q and the location features)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(T, B, N, D1=224, D2=32, F=5, KW=10, seed=0):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g)   # noqa: E731
    return dict(K1=r(B, N, D1) * 0.5, K2=r(B, N, D2) * 0.5, q=r(T, B, D1 + D2) * 0.5,
                b1=r(D1) * 0.1, v1=r(D1), v2=r(D2), locW=r(F, D1) * 0.3, loc=r(T, B, N, F),
                s_prev=torch.rand(T, B, N, generator=g), de1=r(T, B, N), de2=r(T, B, N),
                df=r(T, B, N, F))


def _reference(c, D1, F, KW):
    d = {k: v.double() for k, v in c.items()}
    z1 = torch.tanh(d["K1"][None] + d["q"][:, :, None, :D1] + d["b1"] +
                    torch.einsum("tbnf,fd->tbnd", d["loc"], d["locW"]))
    z2 = torch.tanh(d["K2"][None] + d["q"][:, :, None, D1:])
    dp1 = d["de1"][..., None] * d["v1"] * (1 - z1 * z1)
    dp2 = d["de2"][..., None] * d["v2"] * (1 - z2 * z2)
    out = dict(dK1=dp1.sum(0), dK2=dp2.sum(0),
               dv1=(z1 * d["de1"][..., None]).sum((0, 1, 2)),
               dv2=(z2 * d["de2"][..., None]).sum((0, 1, 2)),
               dWloc=torch.einsum("tbnf,tbnd->fd", d["loc"], dp1))
    # dconvW[j][f] = sum s_{t-1}[n + j - padl] df_t[n][f]; dconvb[f] = sum df_t[n][f]
    T, B, N = d["de1"].shape
    padl = (KW - 1) // 2
    sp = torch.nn.functional.pad(d["s_prev"], (padl, KW - 1 - padl))
    win = torch.stack([sp[..., j:j + N] for j in range(KW)], -1)          # [T, B, N, KW]
    out["dconvW"] = torch.einsum("tbnj,tbnf->jf", win, d["df"])
    out["dconvb"] = d["df"].sum((0, 1, 2))
    return out, z1, z2


@pytest.mark.parametrize("T,B,N,ts", [(7, 2, 13, 1), (33, 3, 200, 1), (500, 2, 61, 1),
                                      (7, 2, 13, 3), (33, 3, 200, 2), (500, 2, 61, 4),
                                      (5, 1, 9, 5)])
def test_attn_param_grads(cuda, T, B, N, ts):
    """sat_attn_param_grads against float64 autograd, unsplit and with the T steps split into
    ts ranges (tsplit; T = ts: one step per range)."""
    from sat_amd import kernels as K
    D1, D2, F, KW = 224, 32, 5, 10
    c = _case(T, B, N, D1, D2, F, KW, seed=T + N)
    ref, _, _ = _reference(c, D1, F, KW)
    dv = {k: v.to(cuda).contiguous() for k, v in c.items()}
    pgs = K.pg_stride(D1, D2, F, KW)
    PG = torch.full((ts * K.attn_param_grad_rows(B, N), pgs), float("nan"), device=cuda)
    dK1s = torch.full((ts, B, N, D1), float("nan"), device=cuda)
    dK2s = torch.full((ts, B, N, D2), float("nan"), device=cuda)
    dK1, dK2 = dK1s[0], dK2s[0]
    q = dv["q"]
    K.attn_param_grads(
        T=T, B=B, N=N, D1=D1, D2=D2, F=F, KW=KW, att1_forward=1, K1=dv["K1"], K2=dv["K2"],
        q=q, q_tstride=q.stride(0), q_bstride=q.stride(1), b1=dv["b1"], v1=dv["v1"],
        locW=dv["locW"], v2=dv["v2"], loc=dv["loc"], s_prev=dv["s_prev"],
        s_tstride=dv["s_prev"].stride(0), de1=dv["de1"], de2=dv["de2"], df=dv["df"],
        dK1=dK1s, dK2=dK2s, pg=PG, pg_stride=pgs, tsplit=ts)
    torch.cuda.synchronize()
    pg = PG.double().cpu().sum(0)
    o = 0
    got = {}
    for name, n in (("dv1", D1), ("dWloc", F * D1), ("dconvW", KW * F), ("dconvb", F),
                    ("dv2", D2)):
        got[name] = pg[o:o + n]
        o += n
    got["dWloc"] = got["dWloc"].view(F, D1)
    got["dconvW"] = got["dconvW"].view(KW, F)
    got["dK1"], got["dK2"] = dK1.double().cpu(), dK2.double().cpu()
    for k, want in ref.items():
        err = float((got[k] - want).abs().max())
        scale = float(want.abs().max()) + 1e-12
        assert err <= 2e-5 * scale * max(1.0, (T / 32) ** 0.5), (k, err, scale)
