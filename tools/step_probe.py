"""Per-launch cost of every decoder-step kernel under hipGraph replay (HIP events).

    python tools/step_probe.py [--batch 32]

Runs one training step for realistic state, then for each kernel type captures T' launches
(one decoder pass) into a graph, replays it, and prints the average time per launch.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import data, engine, hparams, train  # noqa: E402
from sat_amd import kernels as K  # noqa: E402


def timed_graph(fn, Tp, reps=3):
    for t in range(min(Tp, 4)):
        fn(t)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for t in range(Tp):
            fn(t)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * Tp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    B, N, T = a.batch, 200, 1000
    hp = hparams.ljspeech_hparams()
    m = engine.Tacotron(hp, "cuda", pipeline_chunk=0)
    d = m.d
    b = data.synthetic_batch(hp, B, N=N, T=T, shape="max", seed=1)
    batch = {k: torch.tensor(v).cuda() for k, v in b.items()}
    tr = train.Trainer(m, B, N, T // 2)
    tr.forward_backward(batch)
    torch.cuda.synchronize()
    S = tr.last_saved["dec"].tensors
    P = m.P
    Tp = S["Q"].shape[0]
    A, Dd, M1, M2, D1, D2 = d.att_rnn, d.dec, d.m1, d.m2, d.d1, d.d2
    R0 = M1 + M2 + A
    f = dict(device="cuda")
    p_w = S["prenet"][-1].shape[-1]
    W0r = P["decoder/attention_lstm/kernel"][p_w:]
    W1 = P["decoder/lstm1/kernel"]
    ntiles = (N + 31) // 32
    scr = {k: torch.empty(B, 4 * A, **f) for k in ("g", "dg")}
    hs = [torch.zeros(B, A, **f) for _ in range(6)]
    res = {}
    tiny = torch.zeros(4, **f)
    res["empty (axpby 4 floats)"] = timed_graph(lambda t: K.axpby(tiny, tiny, 1.0, 0.0), Tp)
    res["lstm_fwd K=544 (attention RNN)"] = timed_graph(lambda t: K.lstm_step_fwd(
        B=B, U=A, K=R0, t=t, xproj=S["X0"][t], rin=S["REC0"][t], W=W0r, c_prev=S["C0"][t],
        h_prev=S["REC0"][t, :, M1 + M2:], mask_c=None, mask_h=None, zc=0.1, zh=0.1,
        h_raw=hs[0], c_out=hs[1], h_out=hs[2], gates=scr["g"]), Tp)
    res["lstm_fwd K=256 (decoder LSTM)"] = timed_graph(lambda t: K.lstm_step_fwd(
        B=B, U=Dd, K=Dd, t=t, xproj=S["X1"][t], rin=S["H1S"][t], W=W1[A + M1 + M2:],
        c_prev=S["C1S"][t], h_prev=S["H1S"][t], mask_c=None, mask_h=None, zc=0.1, zh=0.1,
        h_raw=hs[0], c_out=hs[1], h_out=hs[2], gates=scr["g"]), Tp)
    QT = torch.empty(D1 + D2, A, **f)
    Qs = torch.empty(B, D1 + D2, **f)
    res["rowdot query [32x256]x[256x256]"] = timed_graph(
        lambda t: K.rowdot(S["H0RAW"][t], QT, Qs), Tp)
    DC = torch.empty(B, M1 + M2, **f)
    res["rowdot dctx [32x1024]x[1024x288]"] = timed_graph(
        lambda t: K.rowdot(S["G0"][t], W0r[:M1 + M2], DC, beta=1.0), Tp)
    pst = K.part_stride(M1, M2)
    E1, E2 = torch.empty(B, N, **f), torch.empty(B, N, **f)
    PART = torch.empty(B, ntiles, pst, **f)
    so, ao, s2o = torch.empty(B, N, **f), torch.empty(B, N, **f), torch.empty(B, N, **f)
    ctx = torch.empty(B, M1 + M2, **f)
    st = torch.empty(B, 4, **f)
    a1 = "decoder/attention1"

    def attn(t, phases, lpp=0):
        K.attn_step_fwd(
            B=B, N=N, D1=D1, M1=M1, D2=D2, M2=M2, F=d.loc_f, KW=d.loc_k, NT=32, ntiles=ntiles,
            att1_forward=1, u=0.5, q=S["Q"][t], q_sb=D1 + D2, K1=S["K1"], V1=S["V1"], K2=S["K2"],
            V2=S["V2"], lengths=batch["source_length"], s_prev=S["S1"][t], a_prev=S["AL1"][t],
            v1=P[f"{a1}/attention_variable"], b1=P[f"{a1}/attention_bias"],
            convW=P[f"{a1}/location_conv/kernel"], convb=P[f"{a1}/location_conv/bias"],
            locW=P[f"{a1}/location_layer/kernel"], v2=P["decoder/attention2/attention_v"],
            e1=E1, e2=E2, part=PART, part_stride=pst, s_out=so, a_out=ao, s2_out=s2o, ctx=ctx,
            ctx_sb=M1 + M2, stats=st, phases=phases, lpp=lpp)
    for lpp in (8, 16, 32):
        res[f"attn fwd energy tile lpp={lpp}"] = timed_graph(lambda t, l=lpp: attn(t, 1, l), Tp)
    res["attn fwd energy + combine (2 launches)"] = timed_graph(lambda t: attn(t, 3), Tp)
    YA = torch.zeros(B, N, **f)
    DF = torch.zeros(B, N, d.loc_f, **f)
    DQ = torch.empty(B, ntiles, D1 + D2, **f)
    DQR = torch.empty(B, D1 + D2, **f)
    DE = torch.empty(B, N, **f)
    DQ8 = torch.empty(B, (N + 7) // 8, D1 + D2, **f)
    dctx = torch.randn(Tp, B, M1 + M2, **f) * 1e-3

    def attn_bwd(t, nt=32, waves=0):
        ntl = (N + nt - 1) // nt
        K.attn_step_bwd(
            B=B, N=N, D1=D1, M1=M1, D2=D2, M2=M2, F=d.loc_f, KW=d.loc_k, NT=nt, ntiles=ntl,
            att1_forward=1, u=0.5, dctx=dctx[t], dctx_sb=M1 + M2, ctx_t=S["REC0"][t + 1],
            ctx_sb=S["REC0"].shape[-1], y_next=YA, V1=S["V1"],
            V2=S["V2"], s_t=S["S1"][t + 1], a_t=S["AL1"][t + 1],
            a_prev=S["AL1"][t], s_prev=S["S1"][t], s2_t=S["S2"][t], stats=S["ST"][t],
            df_next=DF, q=S["Q"][t], q_sb=D1 + D2, K1=S["K1"], K2=S["K2"],
            v1=P[f"{a1}/attention_variable"], b1=P[f"{a1}/attention_bias"],
            convW=P[f"{a1}/location_conv/kernel"], convb=P[f"{a1}/location_conv/bias"],
            locW=P[f"{a1}/location_layer/kernel"], v2=P["decoder/attention2/attention_v"],
            y_out=YA, df_out=DF, de1_out=DE, de2_out=DE, dqp=DQ8, waves=waves)
    for nt, w in ((16, 4), (16, 8), (16, 16), (32, 4), (32, 8), (32, 16)):
        res[f"attn bwd NT={nt} waves={w}"] = timed_graph(
            lambda t, nt=nt, w=w: attn_bwd(t, nt, w), Tp)
    dy = torch.randn(Tp, B, A, **f) * 1e-3

    def lstm_bwd(t, dq):
        K.lstm_step_bwd(B=B, U=A, K=R0, hoff=M1 + M2, t=t, W=W0r, dgates_next=scr["dg"],
                        gates=S["G0"][t], c_prev=S["C0"][t], dy=dy[t], dh_carry=hs[3],
                        dc_carry=hs[4], mask_c=None, mask_h=None, zc=0.1, zh=0.1,
                        dgates=scr["g"], dh_carry_out=hs[5], dc_carry_out=hs[0],
                        **(dict(dq0=DQ[:, :, :D1], wq0=P[f"{a1}/query_layer/kernel"],
                                dq1=DQ[:, :, D1:], wq1=P["decoder/attention2/query_layer/kernel"],
                                dq_parts=ntiles, dq_pstride=D1 + D2,
                                dq_bstride=ntiles * (D1 + D2)) if dq else {}))
    res["lstm_bwd (plain)"] = timed_graph(lambda t: lstm_bwd(t, False), Tp)
    res["lstm_bwd (+ query-gradient partials)"] = timed_graph(lambda t: lstm_bwd(t, True), Tp)

    def lstm_bwd_red(t):
        K.lstm_step_bwd(B=B, U=A, K=R0, hoff=M1 + M2, t=t, W=W0r, dgates_next=scr["dg"],
                        gates=S["G0"][t], c_prev=S["C0"][t], dy=dy[t], dh_carry=hs[3],
                        dc_carry=hs[4], mask_c=None, mask_h=None, zc=0.1, zh=0.1,
                        dgates=scr["g"], dh_carry_out=hs[5], dc_carry_out=hs[0],
                        dq0=DQR[:, :D1], wq0=P[f"{a1}/query_layer/kernel"], dq1=DQR[:, D1:],
                        wq1=P["decoder/attention2/query_layer/kernel"], dq_parts=1,
                        dq_pstride=0, dq_bstride=D1 + D2)
    res["lstm_bwd (+ reduced query gradient)"] = timed_graph(lstm_bwd_red, Tp)
    for k, v in res.items():
        print(f"{k:40s} {v:8.2f} us/launch", flush=True)


if __name__ == "__main__":
    main()
