"""SURVEY.md 8(b)'s single C entries for the decoder loop, called through ctypes:
sat_decoder_loop_fwd == decoder.py decoder_forward's persistent sequence (attention chain launch,
LSTM1 input GEMMs, LSTM stack launch) and sat_decoder_loop_bwd == backward.py decoder_bwd's
(LSTM stack BPTT, LSTM1 input-gradient GEMMs, attention chain BPTT), bit for bit, on the same
inputs.  The reference graph is DecoderRNNV2 (modules/module.py:1531-1540) under
TransformerTrainingHelper (modules/helpers.py:13-58)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


class _Rec:
    """Records the keyword arguments of kernels.<name> while forwarding the call."""

    def __init__(self, K, name):
        self.K, self.name, self.orig, self.kw = K, name, getattr(K, name), None
        setattr(K, name, self)

    def __call__(self, **kw):
        self.kw = dict(kw)
        self.orig(**kw)

    def restore(self):
        setattr(self.K, self.name, self.orig)


def _same(fresh, rec, name):
    """every element the entry wrote (the fresh buffer starts as NaN) equals the launch path's;
    most of the buffer was written (padded positions a kernel never touches may stay NaN)"""
    written = ~torch.isnan(fresh)
    assert float(written.float().mean()) > 0.5, name
    assert torch.equal(fresh[written], rec[written]), name


def _fill(st, kw, fresh):
    from sat_amd import kernels as K
    for k, v in kw.items():
        v = fresh.get(k, v)
        setattr(st, k, K._p(v) if isinstance(v, torch.Tensor) else v)


@pytest.mark.parametrize("B,N,T", [(8, 40, 24), (32, 200, 60)])
def test_decoder_loop_entries_match_python_orchestration(cuda, B, N, T):
    from sat_amd import _lib, data, engine, hparams, params
    from sat_amd import kernels as K
    hp = hparams.ljspeech_hparams()
    vals = params.init_params(hp, seed=5)
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="ljs", seed=3)
    Np, Tp = b["source"].shape[1], b["mel"].shape[1] // hp.outputs_per_step
    mk = data.synthetic_masks(hp, B, Np, Tp, seed=4)
    gb = {k: torch.tensor(v).to(cuda) for k, v in b.items()}
    gm = {k: torch.tensor(v).to(cuda) for k, v in mk.items()}
    m = engine.Tacotron(hp, cuda, init_values=vals, persistent_decoder=True)
    recs = [_Rec(K, n) for n in ("decoder_attention_fwd", "decoder_lstms_fwd",
                                 "decoder_lstms_bwd", "decoder_attention_bwd")]
    try:
        out, sv = m.forward(gb, gm, training=True)
        m.backward(sv)
        torch.cuda.synchronize()
    finally:
        for r in recs:
            r.restore()
    af, lf, lb, ab = (r.kw for r in recs)
    assert all(kw is not None for kw in (af, lf, lb, ab))
    S = sv["dec"].tensors
    lib = _lib.load()
    ws = torch.empty(K.GEMM_WS_BYTES, dtype=torch.uint8, device=cuda)
    W1 = m.P["decoder/lstm1/kernel"]
    A, M1, M2 = af["U"], af["M1"], af["M2"]

    # ---- forward: fresh outputs (row 0 of the state histories = the initial states)
    fresh_a = {k: af[k].clone() for k in ("REC0", "C0", "S1", "AL1")}
    fresh_a.update({k: torch.full_like(af[k], float("nan")) for k in
                    ("H0RAW", "G0", "Q", "S2", "ST", "LOC", "ZH") if af.get(k) is not None})
    fresh_l = {k: lf[k].clone() for k in ("C1S", "H1S", "C2S", "H2S")}
    fresh_l.update({k: torch.full_like(lf[k], float("nan")) for k in
                    ("H1RAW", "G1", "H2RAW", "G2", "X1")})
    for k in ("REC0", "C0", "S1", "AL1"):      # only row 0 is an input
        fresh_a[k][1:] = float("nan")
    for k in ("C1S", "H1S", "C2S", "H2S"):
        fresh_l[k][1:] = float("nan")
    d = _lib.SatDecoderLoopFwd()
    _fill(d.attn, af, fresh_a)
    _fill(d.lstm, lf, fresh_l)
    d.W1x, d.b1 = K._p(W1[:A + M1 + M2]), K._p(m.P["decoder/lstm1/bias"])
    d.ws, d.ws_bytes = K._p(ws), ws.numel()
    _lib.check(lib.sat_decoder_loop_fwd(ctypes.byref(d), K._stream()), "sat_decoder_loop_fwd")
    torch.cuda.synchronize()
    for k in fresh_a:
        _same(fresh_a[k], af[k], k)
    for k in fresh_l:
        _same(fresh_l[k], lf[k], k)

    # ---- backward: fresh gradient outputs, same forward histories and dL/dh2
    fresh_b = {k: torch.full_like(lb[k], float("nan")) for k in ("DG1", "DG2")}
    fresh_c = {k: torch.full_like(ab[k], float("nan")) for k in
               ("DH0", "RD", "DG0", "DE1", "DE2", "DFH", "DQP")}
    db = _lib.SatDecoderLoopBwd()
    _fill(db.lstm, lb, fresh_b)
    _fill(db.attn, ab, fresh_c)
    db.W1x, db.DH0 = K._p(W1[:A + M1 + M2]), K._p(fresh_c["DH0"])
    db.ws, db.ws_bytes = K._p(ws), ws.numel()
    _lib.check(lib.sat_decoder_loop_bwd(ctypes.byref(db), K._stream()), "sat_decoder_loop_bwd")
    torch.cuda.synchronize()
    for k in fresh_b:
        _same(fresh_b[k], lb[k], k)
    for k in fresh_c:
        _same(fresh_c[k], ab[k], k)
    assert int(S["attn_scratch"].err[0]) == 0
