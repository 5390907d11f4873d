"""Hand-written backward (BPTT) of the teacher-forced step, on libsat_hip.

Reverse of ``model.model_forward``: loss seeds -> RNNTransformer head -> decoder LSTM2, LSTM1
recurrences -> attention RNN + dual-source attention recurrence -> memories -> encoder
(self-attention, BiLSTM, highway, CBHG convolutions + BatchNorm, prenets) -> embedding.
Weight gradients ACCUMULATE into the flat gradient arena (``G`` views, zeroed by the caller);
every per-step weight product is deferred to one big MFMA GEMM over all steps after each
recurrence (dW = sum_t x_t^T dgates_t).
"""

from __future__ import annotations

import math
import os
from typing import Dict

import torch

from . import _lib
from . import kernels as K
from .model import _contig_span, bank_fused
from .pipeline import SEQUENTIAL, Pipeline


class Aux:
    """The backward's second stream for weight gradients nothing downstream reads: each branch
    forks from the main stream at its call (so it sees the main stream's operands), runs on
    K.aux_stream, and model_backward joins once after the encoder.  The main stream's dX chain
    is a string of small launches and the encoder BiLSTM BPTT holds 64 CUs, so the branches
    fill idle CUs.  Every tensor a branch reads is referenced until the join (the allocator
    must not hand its block to a later main-stream allocation while the branch may run)."""

    def __init__(self, device):
        self.dev = device
        self.s = K.aux_stream(device)
        self.used = [self.s]
        self.keep = []

    def run(self, fn, *tensors):
        self.s.wait_stream(torch.cuda.current_stream())
        self.keep.extend(tensors)
        with torch.cuda.stream(self.s):
            fn()

    def run_side(self, fn, *tensors, which: int = 2):
        """run a branch on a stream of its own (K.aux_stream index 2, or ``which``), forked here
        from the main stream and joined with the others: it does not queue behind the aux
        backlog"""
        s = K.aux_stream(self.dev, which)
        s.wait_stream(torch.cuda.current_stream())
        if s not in self.used:
            self.used.append(s)
        self.keep.extend(tensors)
        with torch.cuda.stream(s):
            fn()

    def switch(self):
        """Later branches on a further stream, so they do not queue behind the branches issued
        so far (the decoder's weight-gradient backlog)."""
        self.s = K.aux_stream(self.dev, 1)
        self.used.append(self.s)

    def join(self):
        for s in self.used:
            torch.cuda.current_stream().wait_stream(s)
        self.keep.clear()


def _wgrad(aux, fn, *tensors):
    """run a weight-gradient-only product on the aux stream (inline without one)"""
    if aux is not None:
        aux.run(fn, *tensors)
    else:
        fn()


def lin_bwd(x, dy, W, dW, db, ws, dx=None, beta_dx=0.0, need_dx=True, aux=None):
    """Dense backward: dW += x^T dy, db += colsum(dy), dx (=|+=) dy W^T.  x [.., in], dy [.., out].
    With ``aux`` the dW product runs on the aux stream."""
    x2 = x.reshape(-1, x.shape[-1])
    dy2 = dy.reshape(-1, dy.shape[-1])
    wgrad = lambda: K.gemm(x2.t(), dy2, dW, beta=1.0, colsum=db)  # noqa: E731  (+ db, fused)
    if aux is not None:
        aux.run(wgrad, x2, dy2)
    else:
        wgrad()
    if not need_dx:
        return None
    if dx is None:
        dx = torch.empty(*dy.shape[:-1], W.shape[0], device=dy.device)
    K.gemm(dy2, W.t(), dx.reshape(-1, W.shape[0]), beta=beta_dx)
    return dx


# the attention parameter pass's T steps in PG_TSPLIT ranges per position (sat_attn_param_grads
# tsplit): 1600 one-position workgroups at 3 waves per SIMD leave the third residency round
# nearly empty; SAT_PG_TSPLIT=1 is the unsplit A/B arm
PG_TSPLIT = int(os.environ.get("SAT_PG_TSPLIT", "3"))
# SAT_WGRAD_BATCH=1: the decoder LSTM kernels' weight-gradient blocks as one batched launch per
# kernel -- measured slower (13.80 -> 13.96 ms/step: its larger grid crowds out the encoder
# backward's short launches beside it; profiles/r05r_wgrad_batch_ab.txt)
WGRAD_BATCH = os.environ.get("SAT_WGRAD_BATCH", "0") == "1"

# SAT_MHA_WGRAD_AUX=1 runs a multi-head attention's four weight gradients on the aux stream
# (sat_mha_bwd_wgrad after a weight-deferred sat_mha_bwd).  Off: measured +0.45 ms/step for both
# hops (the tail's aux branch is the longer one already) and neutral for the decoder head alone
# (profiles/r05n_mha_wgrad_aux_ab.txt) -- the LSTM stack's BPTT waits for the aux join anyway.
MHA_WGRAD_AUX = os.environ.get("SAT_MHA_WGRAD_AUX", "0") == "1"


def mha_bwd(P, G, scope, s, dy, ws, aux=None):
    """Backward of model.mha_fwd: ONE sat_mha_bwd call.  Returns dx [B, L, W].  With ``aux`` the
    four weight gradients are deferred to sat_mha_bwd_wgrad on the aux stream."""
    names = [f"{scope}/{n}_projection/{t}" for n in ("query", "key", "value", "output")
             for t in ("kernel", "bias")]
    d, scratch = K.mha_desc(s["x"], *(P[n] for n in names), s["heads"], s["causal"], s["mask"], s)
    dx = torch.empty_like(s["x"])
    dyc = K.contiguous(dy)
    d.dy, d.dx = dyc.data_ptr(), dx.data_ptr()
    grads = [G[n].data_ptr() for n in names]
    defer = aux is not None and MHA_WGRAD_AUX and dy.is_cuda
    if not defer:
        d.dWq, d.dbq, d.dWk, d.dbk, d.dWv, d.dbv, d.dWo, d.dbo = grads
    K.mha_bwd(d)
    if defer:
        dw = type(d).from_buffer_copy(d)
        dw.dWq, dw.dbq, dw.dWk, dw.dbk, dw.dWv, dw.dbv, dw.dWo, dw.dbo = grads

        def wgrad():
            wsb = K._gemm_ws(dy.device)        # the aux stream's own split-K scratch
            dw.gemm_ws, dw.gemm_ws_bytes = wsb.data_ptr(), wsb.numel()
            K.mha_bwd_wgrad(dw)
        # the branch reads x, o, dy and the scratch's dQ / dK / dV: referenced until the join
        aux.run(wgrad, scratch, dyc, s["x"], s["o"])
    return dx


def sa_transformer_bwd(P, G, scope, s, dz, ws, aux=None):
    """z = x + tanh(Dense(MHA(x)))  ->  dx."""
    du = torch.empty_like(dz)
    K.act_bwd(dz, s["u"], du, "tanh")
    dy = lin_bwd(s["y"], du, P[f"{scope}/transform/kernel"], G[f"{scope}/transform/kernel"],
                 G[f"{scope}/transform/bias"], ws, aux=aux)
    dx = mha_bwd(P, G, f"{scope}/mha", s, dy, ws, aux=aux)
    K.axpby(dz, dx, 1.0, 1.0)                                        # residual
    return dx


def head_bwd(P, G, hp, d, sv, ws, aux=None):
    """RNNTransformer head backward -> dL/dD step-major [T', B, dec].  With ``aux`` the dense
    layers' weight gradients run on the second stream; the caller joins it before the next
    persistent launch (the LSTM stack's BPTT needs every CU free to become resident)."""
    Z = sv["Z"]
    B, Tp, _ = Z.shape
    dmel_r = sv["dmel"].view(B, Tp, d.num_mels * d.r)
    dstop = sv["dstop"].view(B, Tp, 1)
    dZ = lin_bwd(Z, dmel_r, P["decoder/out_projection/kernel"], G["decoder/out_projection/kernel"],
                 G["decoder/out_projection/bias"], ws, aux=aux)
    lin_bwd(Z, dstop, P["decoder/stop_token_projection/kernel"],
            G["decoder/stop_token_projection/kernel"], G["decoder/stop_token_projection/bias"], ws,
            dx=dZ, beta_dx=1.0, aux=aux)
    dz = dZ
    for h in reversed(range(d.dec_hops)):
        dz = sa_transformer_bwd(P, G, f"decoder/self_attention{h}", sv[f"dec_sa{h}"], dz, ws,
                                aux=aux)
    return K.contiguous(dz.transpose(0, 1))                          # [T', B, D] (data movement)


class _LstmBwd:
    """Reverse recurrence of one LSTM layer, resumable across chunks of steps (the dh/dc carries
    ping-pong between two buffers)."""

    def __init__(self, B, U, dev):
        self.shape, self.dev = (B, U), dev
        self.hc = self.cc = None                  # allocated at the first step (the persistent
        self.first = True                         # paths never take one)
        self.cur = 0

    def desc(self, **kw):
        """kwargs of the next reverse step (carries filled in); advances the carry state."""
        if self.hc is None:
            h0, h1, c0, c1 = K.zeros_group(*([self.shape] * 4), device=self.dev)   # one fill
            self.hc, self.cc = [h0, h1], [c0, c1]
        c = self.cur
        kw.update(dh_carry=None if self.first else self.hc[c],
                  dc_carry=None if self.first else self.cc[c],
                  dh_carry_out=self.hc[1 - c], dc_carry_out=self.cc[1 - c])
        self.first = False
        self.cur = 1 - c
        return kw

    def step(self, **kw):
        K.lstm_step_bwd(**self.desc(**kw))


def decoder_bwd(P, G, hp, d, dsv, dH2, masks, ws, attn_tile=32, pipe: Pipeline = SEQUENTIAL,
                aux: "Aux" = None):
    """Backward of decoder.decoder_forward.  Returns (dm1, dm2) batch-major.

    The three reverse recurrences (LSTM2 -> LSTM1 -> attention RNN) run as the mirror image of the
    forward wavefront (``pipeline.Pipeline``): iteration j holds LSTM2 at step T'-1-j and LSTM1
    C steps behind in ONE multi-problem launch, the attention chain 2C steps behind; the input
    gradients of each chunk (dH1, then dH0 and dctx) are chunk GEMMs issued as soon as the
    producing layer has finished the chunk."""
    S = dsv.tensors
    B, N, Tp = dsv.B, dsv.N, dsv.Tp
    dev = dH2.device
    A, Dd, M1, M2, D1, D2 = d.att_rnn, d.dec, d.m1, d.m2, d.d1, d.d2
    zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
    mk = (lambda n: masks[n]) if masks is not None else (lambda n: None)
    f32 = dict(device=dev, dtype=torch.float32)
    R0 = M1 + M2 + A

    W2, dW2 = P["decoder/lstm2/kernel"], G["decoder/lstm2/kernel"]
    W1, dW1 = P["decoder/lstm1/kernel"], G["decoder/lstm1/kernel"]
    DG2 = torch.empty_like(S["G2"])
    DG1 = torch.empty_like(S["G1"])
    dH1 = torch.empty(Tp, B, Dd, **f32)
    dH0 = torch.empty(Tp, B, A, **f32)
    # [dL/dctx_t | recurrent product of the attention RNN] per step: the per-step row-dot with
    # DG0[t+1] fills both halves at once (the ctx half on top of LSTM1's contribution), so the
    # attention RNN's reverse step only does the query-gradient dot
    # RD and the per-step path's carries (YA, hc, cc below) zeroed by ONE fill
    RD, ya0, ya1, hc0, hc1, cc0, cc1 = K.zeros_group(
        (Tp, B, M1 + M2 + A), (B, N), (B, N), (B, A), (B, A), (B, A), (B, A), device=dev)
    DCTX = RD[:, :, :M1 + M2]
    run2, run1 = _LstmBwd(B, Dd, dev), _LstmBwd(B, Dd, dev)
    m2c, m2h, m1c, m1h = (mk("dec/lstm2/zc"), mk("dec/lstm2/zh"), mk("dec/lstm1/zc"),
                          mk("dec/lstm1/zh"))

    def lstm2_desc(t):
        return run2.desc(B=B, U=Dd, K=Dd, hoff=0, t=t, W=W2[Dd:],
                         dgates_next=DG2[t + 1] if t + 1 < Tp else None, gates=S["G2"][t],
                         c_prev=S["C2S"][t], dy=dH2[t], mask_c=None if m2c is None else m2c[t],
                         mask_h=None if m2h is None else m2h[t], zc=zc, zh=zh, dgates=DG2[t])

    def lstm1_desc(t):
        return run1.desc(B=B, U=Dd, K=Dd, hoff=0, t=t, W=W1[A + M1 + M2:],
                         dgates_next=DG1[t + 1] if t + 1 < Tp else None, gates=S["G1"][t],
                         c_prev=S["C1S"][t], dy=dH1[t], mask_c=None if m1c is None else m1c[t],
                         mask_h=None if m1h is None else m1h[t], zc=zc, zh=zh, dgates=DG1[t])

    def dh1_chunk(a, b):
        n = (b - a) * B
        K.gemm(DG2[a:b].view(n, 4 * Dd), W2[:Dd].t(), dH1[a:b].view(n, Dd))

    def dh0_chunk(a, b):
        n = (b - a) * B
        dg = DG1[a:b].view(n, 4 * Dd)
        if A % 128 == 0:     # dL/dh0' and dL/dctx as the two output blocks of ONE product
            K.gemm(dg, W1[:A + M1 + M2].t(), dH0[a:b].view(n, A),
                   C2=RD[a:b].view(n, R0)[:, :M1 + M2])
        else:
            K.gemm(dg, W1[:A].t(), dH0[a:b].view(n, A))
            K.gemm(dg, W1[A:A + M1 + M2].t(), RD[a:b].view(n, R0)[:, :M1 + M2])

    # ---- attention RNN + dual-source attention recurrence
    W0 = P["decoder/attention_lstm/kernel"]
    dW0 = G["decoder/attention_lstm/kernel"]
    p_w = S["prenet"][-1].shape[-1]
    W0r = W0[p_w:]
    a1, a2 = "decoder/attention1", "decoder/attention2"
    fwd = d.att1 == "forward"
    ntiles = (N + attn_tile - 1) // attn_tile
    DG0 = torch.empty(Tp, B, 4 * A, **f32)
    YA = [ya0, ya1]                                          # alignment-recursion grads
    DFH = torch.empty(Tp, B, N, max(d.loc_f, 1), **f32)     # location-feature gradient history
    DE1 = torch.empty(Tp, B, N, **f32)                      # energy-gradient histories
    DE2 = torch.empty(Tp, B, N, **f32)
    # per-step query gradients: per-tile partials (launch path, 8 x 32 persistent kernel) or
    # fully reduced (one part: the one-utterance-per-8-workgroups BPTT)
    dq_parts = (int(_lib.load().sat_decoder_attention_bwd_dq_parts(B, N))
                if S.get("attn_scratch") is not None else ntiles)
    DQP = torch.empty(Tp, B, dq_parts, D1 + D2, **f32)
    hc = [hc0, hc1]
    cc = [cc0, cc1]
    mc0, mh0 = mk("dec/lstm0/zc"), mk("dec/lstm0/zh")
    chain = {"cur": 0}

    def attention_part(t, cur):
        """Context gradient of step t (through the attention RNN's input at t+1) and the
        dual-source attention backward of step t."""
        last = t == Tp - 1
        if not last:   # [c_t | h_t] through the attention RNN's input at step t+1
            K.rowdot(DG0[t + 1], W0r, RD[t], beta=1.0)
        K.attn_step_bwd(
            B=B, N=N, D1=D1, M1=M1, D2=D2, M2=M2, F=d.loc_f, KW=d.loc_k, NT=attn_tile,
            ntiles=ntiles, att1_forward=1 if fwd else 0, u=0.5, dctx=RD[t],
            dctx_sb=R0, ctx_t=S["REC0"][t + 1], ctx_sb=R0,
            y_next=None if last else YA[cur], V1=S["V1"], V2=S["V2"],
            s_t=S["S1"][t + 1], a_t=S["AL1"][t + 1],
            a_prev=S["AL1"][t], s_prev=S["S1"][t], s2_t=S["S2"][t], stats=S["ST"][t],
            df_next=None if last or not fwd else DFH[t + 1], q=S["Q"][t], q_sb=D1 + D2,
            K1=S["K1"], K2=S["K2"],
            v1=P[f"{a1}/attention_variable"] if fwd else P[f"{a1}/attention_v"],
            b1=P[f"{a1}/attention_bias"] if fwd else None,
            convW=P[f"{a1}/location_conv/kernel"] if fwd else None,
            convb=P[f"{a1}/location_conv/bias"] if fwd else None,
            locW=P[f"{a1}/location_layer/kernel"] if fwd else None,
            v2=P[f"{a2}/attention_v"], y_out=YA[1 - cur], df_out=DFH[t],
            de1_out=DE1[t], de2_out=DE2[t], dqp=DQP[t])

    def lstm0_desc(t, cur):
        """Reverse step t of the attention RNN: recurrent + query gradients in one dot."""
        last = t == Tp - 1
        return dict(B=B, U=A, K=R0, hoff=M1 + M2, t=t, W=W0r, rec=RD[t][:, M1 + M2:],
                    dgates_next=None, gates=S["G0"][t],
                    c_prev=S["C0"][t], dy=dH0[t], dh_carry=None if last else hc[cur],
                    dc_carry=None if last else cc[cur],
                    mask_c=None if mc0 is None else mc0[t],
                    mask_h=None if mh0 is None else mh0[t], zc=zc, zh=zh, dgates=DG0[t],
                    dh_carry_out=hc[1 - cur], dc_carry_out=cc[1 - cur],
                    dq0=DQP[t][:, :, :D1], wq0=P[f"{a1}/query_layer/kernel"],
                    dq1=DQP[t][:, :, D1:], wq1=P[f"{a2}/query_layer/kernel"],
                    dq_parts=ntiles, dq_pstride=D1 + D2, dq_bstride=ntiles * (D1 + D2))

    def attention_step(t):
        """attention part of step t; returns the attention RNN's reverse step t (not launched)."""
        cur = chain["cur"]
        attention_part(t, cur)
        chain["cur"] = 1 - cur
        return lstm0_desc(t, cur)

    scratch = S.get("attn_scratch")
    if scratch is not None:
        if S.get("ZH") is None:
            raise RuntimeError("decoder_bwd: the forward ran without keep_tanh (inference mode)")
        # the forward ran the attention chain as one persistent launch: the decoder LSTMs'
        # reverse recurrences first (both layers in ONE persistent launch, LSTM1 one step
        # behind LSTM2, dL/dh1' formed in-kernel from LSTM2's input rows), their input
        # gradients into the chain as whole-sequence GEMMs, then the attention chain's BPTT as
        # ONE persistent launch (sat_decoder_attention_bwd)
        K.decoder_lstms_bwd(
            B=B, T=Tp, U=Dd, zc=zc, zh=zh, W1r=W1[A + M1 + M2:], W2=W2, G1=S["G1"],
            C1S=S["C1S"], G2=S["G2"], C2S=S["C2S"], DH2=dH2, mask1_c=m1c, mask1_h=m1h,
            mask2_c=m2c, mask2_h=m2h, DG1=DG1, DG2=DG2, ctr=scratch.lstm_ctr,
            err=scratch.lstm_err[1])
        dh0_chunk(0, Tp)
        sb = scratch.bwd
        K.decoder_attention_bwd(
            B=B, N=N, T=Tp, U=A, M1=M1, M2=M2, D1=D1, D2=D2, F=d.loc_f, KW=d.loc_k, u=0.5,
            zc=zc, zh=zh, REC0=S["REC0"], C0=S["C0"], G0=S["G0"], S1=S["S1"],
            AL1=S["AL1"], S2=S["S2"], ST=S["ST"], LOC=S["LOC"], V1=S["V1"], V2=S["V2"],
            v1=P[f"{a1}/attention_variable"], convW=P[f"{a1}/location_conv/kernel"],
            convb=P[f"{a1}/location_conv/bias"], locW=P[f"{a1}/location_layer/kernel"],
            v2=P[f"{a2}/attention_v"], W0r=W0r,
            Wq1=P[f"{a1}/query_layer/kernel"], Wq2=P[f"{a2}/query_layer/kernel"],
            mask_c=mc0, mask_h=mh0, DH0=dH0, ZH=S["ZH"], RD=RD, DG0=DG0, DE1=DE1, DE2=DE2, DFH=DFH,
            DQP=DQP, RDP=sb.RDP, YA=sb.YA, ctr=sb.ctr, err=sb.err)
    elif not pipe.enabled:          # layer by layer
        for t in range(Tp - 1, -1, -1):
            K.lstm_step_bwd(**lstm2_desc(t))
        dh1_chunk(0, Tp)
        for t in range(Tp - 1, -1, -1):
            K.lstm_step_bwd(**lstm1_desc(t))
        dh0_chunk(0, Tp)
        for t in range(Tp - 1, -1, -1):
            K.lstm_step_bwd(**attention_step(t))
    else:
        # reverse wavefront: LSTM1 C and the attention chain 2C behind LSTM2.  Iteration j
        # issues ONE multi-problem launch {LSTM2 at T'-1-j, LSTM1 C behind, the attention RNN's
        # step deferred from the previous iteration}, then the attention backward 2C behind.
        C = pipe.chunk
        dh1_at = pipe.finishing_rev(Tp, 0)
        dh0_at = pipe.finishing_rev(Tp, C)
        pending = None
        for j in range(Tp + 2 * C + 1):
            t2, t1, t0 = Tp - 1 - j, Tp - 1 - j + C, Tp - 1 - j + 2 * C
            steps = []
            if t2 >= 0:
                steps.append(lstm2_desc(t2))
            if 0 <= t1 < Tp:
                steps.append(lstm1_desc(t1))
            if pending is not None:
                steps.append(pending)
                pending = None
            if steps:
                K.lstm_steps_bwd(steps)
            if 0 <= t0 < Tp:
                pending = attention_step(t0)
            if j in dh1_at:
                dh1_chunk(*dh1_at[j])
            if j in dh0_at:
                dh0_chunk(*dh0_at[j])
        assert pending is None
    # ---- weight gradients nothing downstream reads -- the LSTM stack's and the attention RNN's
    #      dW, the decoder prenets, the query layers -- run on the aux stream, concurrently with
    #      the attention parameter pass and the encoder backward (which leave CUs idle: the
    #      encoder BiLSTM BPTT holds 64 of them); model_backward joins the stream.  Everything the
    #      branch reads stays referenced until the join; it writes only its own gradient rows.
    aux_s = aux.s if aux is not None else torch.cuda.current_stream()
    # the branch forks after the attention parameter pass is issued (so it waits for it: the
    # pass, on the critical path, no longer shares the chip with these products; 14.86 -> 14.83
    # ms/step, two rounds on one box); SAT_DEC_WGRAD_FORK=bptt forks it at the BPTT (A/B)
    late = os.environ.get("SAT_DEC_WGRAD_FORK", "pg") == "pg"

    def fork_wgrad():
        if aux is not None:
            aux.s.wait_stream(torch.cuda.current_stream())
            aux.keep.extend([DG0, DG1, DG2, DQP, S])
        with torch.cuda.stream(aux_s):
            dec_wgrad()

    def dec_wgrad():
        # LSTM weight gradients: one GEMM per weight block over all steps
        DG2f = DG2.view(Tp * B, 4 * Dd)
        DG1f = DG1.view(Tp * B, 4 * Dd)
        h2s = S["H2S"][:Tp].reshape(Tp * B, Dd)
        h1raw = S["H1RAW"].view(Tp * B, Dd)
        h1s = S["H1S"][:Tp].reshape(Tp * B, Dd)
        h0raw = S["H0RAW"].view(Tp * B, A)
        if WGRAD_BATCH:
            # (A/B only, WGRAD_BATCH above)
            K.gemm_wgrad_batch([h1raw, h2s], DG2f, [dW2[:Dd], dW2[Dd:]],
                               colsum=G["decoder/lstm2/bias"])
            if A == Dd:
                K.gemm_wgrad_batch([h1s, h0raw], DG1f, [dW1[A + M1 + M2:], dW1[:A]],
                                   colsum=G["decoder/lstm1/bias"])
            else:
                K.gemm(h1s.t(), DG1f, dW1[A + M1 + M2:], beta=1.0, colsum=G["decoder/lstm1/bias"])
                K.gemm(h0raw.t(), DG1f, dW1[:A], beta=1.0)
        else:
            K.gemm(h2s.t(), DG2f, dW2[Dd:], beta=1.0)
            K.gemm(h1raw.t(), DG2f, dW2[:Dd], beta=1.0,
                   colsum=G["decoder/lstm2/bias"])                 # + the bias gradient
            K.gemm(h1s.t(), DG1f, dW1[A + M1 + M2:], beta=1.0, colsum=G["decoder/lstm1/bias"])
            K.gemm(h0raw.t(), DG1f, dW1[:A], beta=1.0)
        ctx_all = S["REC0"][1:].reshape(Tp * B, R0)[:, :M1 + M2]
        K.gemm(ctx_all.t(), DG1f, dW1[A:A + M1 + M2], beta=1.0)

        DG0f = DG0.view(Tp * B, 4 * A)
        K.gemm(S["REC0"][:Tp].reshape(Tp * B, R0).t(), DG0f, dW0[p_w:], beta=1.0)
        dP = lin_bwd(S["prenet"][-1], DG0, W0[:p_w], dW0[:p_w], G["decoder/attention_lstm/bias"], ws)
        # decoder prenets (inputs are teacher frames: no input gradient needed for the first one)
        pres = S["prenet"]
        ms = S.get("ms_prenet")
        for i in reversed(range(len(d.dec_prenet))):
            y = pres[i + 1]
            dpre = torch.empty_like(y)
            K.act_bwd(dP, y, dpre, "relu", mask=mk(f"dec/prenet{i}"))
            sc = "decoder/prenet0/dense" if (ms is not None and i == 0) else f"decoder/prenet{i}"
            dP = lin_bwd(pres[i], dpre, P[f"{sc}/kernel"], G[f"{sc}/kernel"], G[f"{sc}/bias"], ws,
                         need_dx=i > 0 or ms is not None)
        if ms is not None:
            multi_speaker_prenet_bwd(P, G, d, S, ms, dP, ws)

        # the per-tile partials of every step sum into the query-layer kernels; the attention bias
        # gradient (the column sum of every tile) rides on each tile's GEMM as its fused colsum row
        H0f = S["H0RAW"].view(Tp * B, A)
        DQt = DQP.view(Tp * B, dq_parts, D1 + D2)
        for tile in range(dq_parts):
            K.gemm(H0f.t(), DQt[:, tile, :D1], G[f"{a1}/query_layer/kernel"], beta=1.0,
                   colsum=G[f"{a1}/attention_bias"] if fwd else None)
            K.gemm(H0f.t(), DQt[:, tile, D1:], G[f"{a2}/query_layer/kernel"], beta=1.0)

    if not late:
        fork_wgrad()
    # ---- attention parameters: one pass over all steps (sat_attn_param_grads), then a column
    #      sum of its per-workgroup partial rows
    F, KW = (d.loc_f, d.loc_k) if fwd else (0, 0)
    pgs = K.pg_stride(D1, D2, F, KW)
    ts = max(1, min(PG_TSPLIT, Tp, 8))     # the library takes 1 <= tsplit <= min(T', 8)
    PG = torch.empty(ts * K.attn_param_grad_rows(B, N), pgs, **f32)
    dK1s = torch.empty(ts, B, N, D1, **f32)       # slab 0 holds the gradient on return
    dK2s = torch.empty(ts, B, N, D2, **f32)
    dK1, dK2 = dK1s[0], dK2s[0]
    Qh = S["Q"]
    K.attn_param_grads(
        T=Tp, B=B, N=N, D1=D1, D2=D2, F=F, KW=KW, att1_forward=1 if fwd else 0,
        K1=S["K1"], K2=S["K2"], q=Qh, q_tstride=Qh.stride(0), q_bstride=Qh.stride(1),
        b1=P[f"{a1}/attention_bias"] if fwd else None,
        v1=P[f"{a1}/attention_variable"] if fwd else P[f"{a1}/attention_v"],
        locW=P[f"{a1}/location_layer/kernel"] if fwd else None, v2=P[f"{a2}/attention_v"],
        loc=S["LOC"] if fwd else None, s_prev=S["S1"], s_tstride=S["S1"].stride(0),
        de1=DE1, de2=DE2, df=DFH if fwd else None, dK1=dK1s, dK2=dK2s, pg=PG, pg_stride=pgs,
        tsplit=ts)
    if late:
        fork_wgrad()
    if fwd:
        dsts = [G[f"{a1}/attention_variable"], G[f"{a1}/location_layer/kernel"].view(-1),
                G[f"{a1}/location_conv/kernel"].view(-1), G[f"{a1}/location_conv/bias"]]
    else:
        dsts = [G[f"{a1}/attention_v"]]
    K.colsum_scatter(PG, dsts + [G[f"{a2}/attention_v"]], ws, beta=1.0)
    # ---- memories: values via the alignment histories, keys via memory_layer
    dV1 = K.gemm(S["AL1"][1:].permute(1, 2, 0), DCTX[:, :, :M1].permute(1, 0, 2))   # [B, N, M1]
    dV2 = K.gemm(S["S2"].permute(1, 2, 0), DCTX[:, :, M1:].permute(1, 0, 2))        # [B, N, M2]
    lin_bwd(S["V1"], dK1, P[f"{a1}/memory_layer/kernel"], G[f"{a1}/memory_layer/kernel"], None,
            ws, dx=dV1, beta_dx=1.0)
    lin_bwd(S["V2"], dK2, P[f"{a2}/memory_layer/kernel"], G[f"{a2}/memory_layer/kernel"], None,
            ws, dx=dV2, beta_dx=1.0)
    return dV1, dV2          # caller applies the sequence mask (values were masked memories)


def multi_speaker_prenet_bwd(P, G, d, S, ms, dd0, ws):
    """Backward of MultiSpeakerPreNet's first stage (modules/multi_speaker_modules.py:27-29):
    d0 = relu(x W0 + b0) + softsign(spk Ws + bs), spk = speaker_embedding[id - offset].
    The speaker row's gradient is the sum of dd0 over the T' steps (a column sum of the
    step-major [T', B*p0] view)."""
    Tp, B, p0 = dd0.shape
    sc = "decoder/prenet0"
    dsp = torch.empty(B, p0, device=dd0.device)
    K.colsum(dd0.view(Tp, B * p0), dsp.view(-1), ws, beta=0.0)
    dspre = torch.empty_like(dsp)
    K.act_bwd(dsp, ms["sp"], dspre, "softsign")
    dspk = lin_bwd(ms["spk"], dspre, P[f"{sc}/speaker_projection/kernel"],
                   G[f"{sc}/speaker_projection/kernel"], G[f"{sc}/speaker_projection/bias"], ws)
    K.embedding_bwd(dspk, ms["ids"], G["speaker_embedding"], offset=d.spk_offset)
    dpre0 = torch.empty_like(dd0)
    K.act_bwd(dd0, ms["y0"], dpre0, "relu")
    lin_bwd(S["xin"], dpre0, P[f"{sc}/dense0/kernel"], G[f"{sc}/dense0/kernel"],
            G[f"{sc}/dense0/bias"], ws, need_dx=False)


def encoder_bwd(P, G, hp, d, sv, dm1, dm2, lengths, masks, ws, aux: Aux = None):
    dev = dm1.device
    mk = (lambda n: masks[n]) if masks is not None else (lambda n: None)
    B, N, _ = dm1.shape
    training = sv["training"]
    # encoder self-attention hops
    dz = dm2
    for h in reversed(range(d.enc_hops)):
        dz = sa_transformer_bwd(P, G, f"encoder/self_attention{h}", sv[f"enc_sa{h}"], dz, ws,
                                aux=aux)
    lin_bwd(sv["m1"], dz, P["encoder/self_attention_projection/kernel"],
            G["encoder/self_attention_projection/kernel"],
            G["encoder/self_attention_projection/bias"], ws, dx=dm1, beta_dx=1.0, aux=aux)
    # BiLSTM
    U = d.cbhg_half
    hws = sv["hws"]
    hw = hws[-1][2] if len(hws) > 1 else hws[0]
    Win = hw.shape[-1]
    hw_box = []

    def hw_sm_of():
        # [N, B, Win] (data movement) for the input-weight gradients, made on the stream that
        # runs them (the aux stream when present: off the main stream's chain)
        if not hw_box:
            hw_box.append(K.contiguous(hw.transpose(0, 1)))
        return hw_box[0]
    dhw = torch.empty(B, N, Win, device=dev)
    zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
    # reverse recurrences of both directions, one multi-problem launch per step (the forward
    # cell walks n = N-1 .. 0, the backward cell n = 0 .. N-1)
    dirs = (("fw", False), ("bw", True))
    DGs = {dr: torch.empty_like(sv["enc_lstm"][dr]["G"]) for dr, _ in dirs}
    runs = {dr: _LstmBwd(B, U, dev) for dr, _ in dirs}

    def enc_bwd_desc(dr, rev, n):
        st = sv["enc_lstm"][dr]
        half = slice(U, 2 * U) if rev else slice(0, U)
        nt = (n - 1 if n > 0 else None) if rev else (n + 1 if n + 1 < N else None)
        mc, mh = mk(f"enc/lstm_{dr}/zc"), mk(f"enc/lstm_{dr}/zh")
        return runs[dr].desc(
            B=B, U=U, K=U, hoff=0, t=n, W=P[f"encoder/cbhg/lstm_{dr}/kernel"][Win:],
            dgates_next=None if nt is None else DGs[dr][nt], gates=st["G"][n],
            c_prev=st["CS"][n + 1] if rev else st["CS"][n], dy=dm1[:, n, half],
            mask_c=None if mc is None else mc[n], mask_h=None if mh is None else mh[n],
            zc=zc, zh=zh, dgates=DGs[dr][n], lengths=lengths)

    if sv.get("enc_persistent"):
        # both directions' reverse recurrences in ONE launch (encoder_lstm.hip)
        mcs = {dr: (mk(f"enc/lstm_{dr}/zc"), mk(f"enc/lstm_{dr}/zh")) for dr, _ in dirs}
        K.encoder_lstm_bwd(
            B=B, N=N, U=U, zc=zc, zh=zh,
            W_fw=P["encoder/cbhg/lstm_fw/kernel"][Win:], W_bw=P["encoder/cbhg/lstm_bw/kernel"][Win:],
            G_fw=sv["enc_lstm"]["fw"]["G"], G_bw=sv["enc_lstm"]["bw"]["G"],
            CS_fw=sv["enc_lstm"]["fw"]["CS"], CS_bw=sv["enc_lstm"]["bw"]["CS"],
            mc_fw=mcs["fw"][0], mh_fw=mcs["fw"][1], mc_bw=mcs["bw"][0], mh_bw=mcs["bw"][1],
            lengths=lengths, DY=dm1, dy_sb=dm1.stride(0), dy_sn=dm1.stride(1),
            DG_fw=DGs["fw"], DG_bw=DGs["bw"])
    else:
        for i in range(N):
            K.lstm_steps_bwd([enc_bwd_desc("fw", False, N - 1 - i), enc_bwd_desc("bw", True, i)])
    for dr, rev in dirs:
        st = sv["enc_lstm"][dr]
        dWk = G[f"encoder/cbhg/lstm_{dr}/kernel"]
        DG = DGs[dr]
        DGf = DG.view(N * B, 4 * U)
        hprev = st["HS"][1:N + 1] if rev else st["HS"][:N]

        def wgrad(hprev=hprev, DGf=DGf, dWk=dWk, dr=dr):
            K.gemm(hprev.reshape(N * B, U).t(), DGf, dWk[Win:], beta=1.0)
            hs = hw_sm_of()
            K.gemm(hs.view(N * B, Win).t(), DGf, dWk[:Win], beta=1.0,
                   colsum=G[f"encoder/cbhg/lstm_{dr}/bias"])      # + the bias gradient
            if aux is not None:
                aux.keep.append(hs)
        if aux is not None:
            aux.run(wgrad, hprev, DGf, hw)
        else:
            wgrad()
    # dhw[b, n, :] = DG_fw[n, b, :] @ Wx_fw^T + DG_bw[n, b, :] @ Wx_bw^T -- batched over n,
    # written transposed, both directions as the two segments of ONE reduction
    (dr0, _), (dr1, _) = dirs
    K.gemm(DGs[dr0], P[f"encoder/cbhg/lstm_{dr0}/kernel"][:Win].t(), dhw.transpose(0, 1),
           A2=DGs[dr1], B2=P[f"encoder/cbhg/lstm_{dr1}/kernel"][:Win].t())
    # highway stack
    dy = dhw
    for i in reversed(range(d.num_highway)):
        h, t, y = hws[i + 1]
        x = hws[i] if i == 0 else hws[i][2]
        dh_pre = torch.empty_like(h)
        dt_pre = torch.empty_like(t)
        dx = torch.empty_like(x)
        K.highway_bwd(h, t, x, dy, dh_pre, dt_pre, dx)
        sc = f"encoder/cbhg/highway{i}"
        WH, WT = P[f"{sc}/H/kernel"], P[f"{sc}/T/kernel"]
        lin_bwd(x, dh_pre, WH, G[f"{sc}/H/kernel"], G[f"{sc}/H/bias"], ws, need_dx=False, aux=aux)
        lin_bwd(x, dt_pre, WT, G[f"{sc}/T/kernel"], G[f"{sc}/T/bias"], ws, need_dx=False, aux=aux)
        # dx += dh_pre W_H^T + dt_pre W_T^T as ONE reduction (two-segment operands)
        w_in = x.shape[-1]
        K.gemm(dh_pre.reshape(-1, WH.shape[1]), WH.t(), dx.reshape(-1, w_in), beta=1.0,
               A2=dt_pre.reshape(-1, WT.shape[1]), B2=WT.t())
        dy = dx
    if d.needs_adjust:
        dy = lin_bwd(sv["hw_in_adjust"], dy, P["encoder/cbhg/adjustment/kernel"],
                     G["encoder/cbhg/adjustment/kernel"], G["encoder/cbhg/adjustment/bias"], ws)
    # proj2: hw0 = BN(p2_pre) + inp
    inp = sv["enc_pre"][-1]
    C2 = d.proj2
    dinp = K.copy3d_(torch.empty_like(dy), dy)                       # residual branch
    dp2 = torch.empty_like(sv["p2_pre"])
    s2 = sv["st_p2"]
    K.bn_bwd(dy.view(-1, C2), sv["p2_pre"].view(-1, C2), None, dp2.view(-1, C2), s2["mean"],
             s2["var"], s2["gamma"], G["encoder/cbhg/proj2/bn/gamma"],
             G["encoder/cbhg/proj2/bn/beta"], ws, training=training)
    # the two projections' weight gradients run after the conv bank's weight gradient on its
    # side stream instead of forking here, where they held the CUs the dX chain's short BN /
    # max-pool launches wait for (a 96 us column-sum finish behind a 127 us GEMM):
    # 14.03 -> 13.99 ms/step, 3 interleaved rounds (profiles/r05q_tail_ab.txt);
    # SAT_PROJ_DW_BANK=0 forks them here again
    proj_later = (aux is not None and bank_fused(d, inp)
                  and os.environ.get("SAT_BANK_DW_SIDE", "1") == "1"
                  and os.environ.get("SAT_PROJ_DW_BANK", "1") == "1")
    # SAT_PROJ_DW_SIDE2=1: those two products on a third side stream forked with the bank's
    # (beside the bank dX and dW products) instead of queued behind the bank dW
    proj_side2 = proj_later and os.environ.get("SAT_PROJ_DW_SIDE2", "0") == "1"
    later = []

    def proj_wgrad(fn, *tensors):
        if proj_later:
            later.append(fn)
            aux.keep.extend(tensors)
        else:
            _wgrad(aux, fn, *tensors)
    proj_wgrad(lambda: (K.conv1d_dw(sv["p1"], dp2, G["encoder/cbhg/proj2/kernel"], beta=1.0),
                        K.colsum(dp2.view(-1, C2), G["encoder/cbhg/proj2/bias"], ws)),
               sv["p1"], dp2)
    dp1 = K.conv1d_dx(dp2, P["encoder/cbhg/proj2/kernel"])
    # proj1: p1 = relu(BN(p1_pre))
    C1 = d.proj1
    dp1_pre = torch.empty_like(dp1)
    s1 = sv["st_p1"]
    K.bn_bwd(dp1.view(-1, C1), sv["p1_pre"].view(-1, C1), sv["p1"].view(-1, C1),
             dp1_pre.view(-1, C1), s1["mean"], s1["var"], s1["gamma"],
             G["encoder/cbhg/proj1/bn/gamma"], G["encoder/cbhg/proj1/bn/beta"], ws,
             training=training)
    proj_wgrad(lambda: (K.conv1d_dw(sv["mp"], dp1_pre, G["encoder/cbhg/proj1/kernel"], beta=1.0),
                        K.colsum(dp1_pre.view(-1, C1), G["encoder/cbhg/proj1/bias"], ws)),
               sv["mp"], dp1_pre)
    dmp = K.conv1d_dx(dp1_pre, P["encoder/cbhg/proj1/kernel"])
    # max-pool, conv bank BN (one launch over the concatenated channels), conv bank
    dbank = torch.empty_like(dmp)
    K.maxpool2_bwd(sv["bank"], dmp, dbank)
    C, KC = d.conv_ch, d.max_k * d.conv_ch
    names = [f"encoder/cbhg/conv_bank/K{k}" for k in range(1, d.max_k + 1)]
    sb = sv["st_bank"]
    dbank_pre = torch.empty_like(dbank)
    K.bn_bwd(dbank.view(-1, KC), sv["bank_pre"].view(-1, KC), sv["bank"].view(-1, KC),
             dbank_pre.view(-1, KC), sb["mean"], sb["var"], sb["gamma"],
             _contig_span(G, [f"{n}/bn/gamma" for n in names]),
             _contig_span(G, [f"{n}/bn/beta" for n in names]), ws, training=training)
    # the conv bank's bias sum rides with its weight gradient on the side stream (it is 0.1 ms
    # of the dX chain otherwise): 14.50 -> 14.48 ms/step, 5 of 5 interleaved pairs; the proj1 /
    # proj2 weight gradients moved there too measured no further gain
    bank_bias = lambda: K.colsum(dbank_pre.view(-1, KC),  # noqa: E731
                                 _contig_span(G, [f"{n}/bias" for n in names]), ws)
    bias_side = (bank_fused(d, inp) and aux is not None
                 and os.environ.get("SAT_BANK_DW_SIDE", "1") == "1"
                 and os.environ.get("SAT_BANK_BIAS_SIDE", "1") == "1")
    if not bias_side:
        bank_bias()
    if bank_fused(d, inp):
        kern = [f"{n}/kernel" for n in names]
        # the weight-gradient branch forks BEFORE the dX product is issued: a branch waits for
        # everything the main stream has issued at its fork, so the other order serialises them
        # the weight-gradient product on a stream of its own (not behind the aux backlog): the
        # graph then runs it beside the dX product instead of before it on the same queue
        # (14.52 -> 14.47 ms/step, 6 interleaved pairs; SAT_BANK_DW_SIDE=0 restores the aux branch)
        bank_dw = lambda: K.conv_bank_bwd(inp, _contig_span(P, kern), dbank_pre,  # noqa: E731
                                          d.max_k, C, dW=_contig_span(G, kern), beta_dw=1.0)
        if aux is not None and os.environ.get("SAT_BANK_DW_SIDE", "1") == "1":
            side = (lambda: (bank_bias(), bank_dw())) if bias_side else bank_dw
            if proj_side2 and later:
                aux.run_side(side, inp, dbank_pre)
                aux.run_side(lambda: [f() for f in later], which=3)
            else:
                aux.run_side((lambda: (side(), [f() for f in later])) if later else side,
                             inp, dbank_pre)
        else:
            _wgrad(aux, bank_dw, inp, dbank_pre)
        K.conv_bank_bwd(inp, _contig_span(P, kern), dbank_pre, d.max_k, C, dx=dinp,
                        beta_dx=1.0)
    else:
        for k in range(1, d.max_k + 1):
            sl = dbank_pre[:, :, (k - 1) * C:k * C]
            K.conv1d_dw(inp, sl, G[f"{names[k - 1]}/kernel"], beta=1.0)
            K.conv1d_dx(sl, P[f"{names[k - 1]}/kernel"], out=dinp, beta=1.0)
    # prenets + embedding
    pre = sv["enc_pre"]
    dx = dinp
    for i in reversed(range(len(d.enc_prenet))):
        y = pre[i + 1]
        dpre = torch.empty_like(y)
        K.act_bwd(dx, y, dpre, "relu", mask=mk(f"enc/prenet{i}"))
        dx = lin_bwd(pre[i], dpre, P[f"encoder/prenet{i}/kernel"], G[f"encoder/prenet{i}/kernel"],
                     G[f"encoder/prenet{i}/bias"], ws, aux=aux)
    K.embedding_bwd(dx, sv["batch"]["source"], G["embedding"])


def model_backward(P, G, hp, d, sv, ws, attn_tile=32, pipe: Pipeline = SEQUENTIAL,
                   on_decoder_grads=None):
    """Accumulate dL/dparams of model_forward's loss into G (caller zeroes G).

    ``on_decoder_grads(streams)``: called once every decoder-side gradient (the speaker
    embedding, prenets, attention RNN and mechanisms, LSTM stack, head, projections -- the
    arena's tail behind the encoder, ``Tacotron.decoder_grad_span``) has been ISSUED, before the
    encoder's backward starts; ``streams`` are the streams that carry that work (the caller
    waits on them, e.g. to all-reduce that bucket beside the encoder backward).  The encoder
    backward writes only encoder / embedding rows (``encoder_bwd``)."""
    masks = sv["masks"]
    aux = Aux(sv["Z"].device) if sv["Z"].is_cuda else None
    dH2 = head_bwd(P, G, hp, d, sv, ws, aux=aux)
    if aux is not None:
        aux.join()        # before the LSTM stack's BPTT (persistent: all 256 workgroups resident)
    dV1, dV2 = decoder_bwd(P, G, hp, d, sv["dec"], dH2, masks, ws, attn_tile=attn_tile,
                           pipe=pipe, aux=aux)
    lengths = sv["batch"]["source_length"]
    dm1 = K.seq_mask(dV1, lengths)
    dm2 = K.seq_mask(dV2, lengths)
    if on_decoder_grads is not None:
        on_decoder_grads([torch.cuda.current_stream()] + (list(aux.used) if aux is not None
                                                          else []))
    if aux is not None and os.environ.get("SAT_AUX2") == "1":
        aux.switch()      # A/B: the encoder's weight-gradient branches on their own stream
    encoder_bwd(P, G, hp, d, sv, dm1, dm2, lengths, masks, ws, aux=aux)
    if aux is not None:
        aux.join()                                    # every weight-gradient branch