"""DualSourceTransformerDecoder teacher-forced loop on libsat_hip (forward).

Mirrors ``DualSourceTransformerDecoder.call`` (modules/module.py:1499-1562) with
``RNNTransformer``'s training branch (:743-747): ``dynamic_decode`` over T' = T/r steps of
``DecoderRNNV2 = MultiRNNCell([DualSourceAttentionRNN, ZoneoutLSTM, ZoneoutLSTM])``.

MI355X restructuring (same arithmetic, different schedule):
* teacher forcing makes every decoder input known up front, so the prenets and every LSTM's
  input projection (x @ W_x + b) are hoisted out of the recurrence into large MFMA GEMMs;
* the recurrence of the attention RNN (ZoneoutLSTM 256 -> query -> dual-source attention) runs
  first over all steps: 3 launches per step (LSTM step, query GEMV, attention tile+combine);
* the two decoder LSTMs depend only on the attention RNN's outputs, so they run as a wavefront
  behind it (``pipeline.Pipeline``): ONE multi-problem launch per iteration holds the attention
  RNN at step i, LSTM1 at i - C and LSTM2 at i - 2C, with the LSTMs' input GEMMs hoisted per
  chunk of C steps.  Per decoder step: 3 launches for the attention chain, none extra for the
  two decoder LSTMs.

All state histories are kept (step-major ``[T'+1, B, .]``) for the hand-written BPTT.
"""

from __future__ import annotations

import warnings
from dataclasses import dataclass, field
from typing import Dict, Optional

import torch

from . import kernels as K
from .params import Dims
from .pipeline import SEQUENTIAL, Pipeline


@dataclass
class DecoderSaved:
    B: int
    N: int
    Tp: int
    tensors: Dict[str, torch.Tensor] = field(default_factory=dict)

    def __getattr__(self, k):
        t = self.__dict__.get("tensors", {})
        if k in t:
            return t[k]
        raise AttributeError(k)


def teacher_inputs(targets: torch.Tensor, r: int, n_feed: int) -> torch.Tensor:
    """TransformerTrainingHelper (modules/helpers.py:44-58): step 0 = go frame (zeros),
    step t = targets.reshape(B, T/r, M*r)[:, t-1, -M*n_feed:].  Step-major [T', B, M*n_feed];
    pure data movement."""
    B, T, M = targets.shape
    Tp = T // r
    x = torch.empty(Tp, B, M * n_feed, device=targets.device, dtype=targets.dtype)
    g = targets.view(B, Tp, M * r)
    K.fill_(x[0])
    K.copy3d_(x[1:], g[:, :-1, M * (r - n_feed):].transpose(0, 1))
    return x


def _state_shapes(d: Dims, Tp: int, B: int, N: int):
    """zero-initialised state histories (row 0 = initial state) of the attention RNN and the
    decoder LSTMs: REC0 [c1 | c2 | h0], C0, S1, AL1, c1, h1, c2, h2"""
    A, Dd = d.att_rnn, d.dec
    R0 = d.m1 + d.m2 + A
    return ((Tp + 1, B, R0), (Tp + 1, B, A), (Tp + 1, B, N), (Tp + 1, B, N),
            (Tp + 1, B, Dd), (Tp + 1, B, Dd), (Tp + 1, B, Dd), (Tp + 1, B, Dd))


def decoder_inputs(P: Dict[str, torch.Tensor], hp, d: Dims, targets: torch.Tensor,
                   masks: Optional[Dict[str, torch.Tensor]], aux,
                   N: Optional[int] = None) -> Dict[str, object]:
    """The part of the teacher-forced decoder that reads only the targets (single speaker):
    teacher frames, the prenets (dropout fused) and the attention RNN's input projection of the
    prenet part.  Every output is allocated on the CURRENT stream, then the products run on the
    stream ``aux`` (forked from the current one); the caller joins ``aux`` before
    decoder_forward(inputs=...) reads them.  With ``N`` (encoder positions) the decoder's zeroed
    state histories are made on ``aux`` too ("hist"), off the encoder's critical path."""
    r, nf = d.r, hp.n_feed_frame
    B, T, M = targets.shape
    Tp = T // r
    dev = targets.device
    mk = (lambda name: masks[name]) if masks is not None else (lambda name: None)
    xin = torch.empty(Tp, B, M * nf, device=dev, dtype=targets.dtype)
    pres = [xin] + [torch.empty(Tp, B, w, device=dev) for w in d.dec_prenet]
    X0 = torch.empty(Tp, B, 4 * d.att_rnn, device=dev)
    hist = K.empty_group(*_state_shapes(d, Tp, B, N), device=dev) if N is not None else None
    aux.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(aux):
        if hist is not None:
            K.fill_(hist[0])
            K.copy3d_(hist[1][3][0, :, 0:1], K.ones(B, 1, device=dev))   # AL1 row 0
            #                                                  (forward_attention.py:131-133)
        g = targets.view(B, Tp, M * r)
        K.fill_(xin[0])                                  # the go frame
        K.copy3d_(xin[1:], g[:, :-1, M * (r - nf):].transpose(0, 1))
        for i in range(len(d.dec_prenet)):
            K.linear(pres[i], P[f"decoder/prenet{i}/kernel"], P[f"decoder/prenet{i}/bias"],
                     act="relu", mul=mk(f"dec/prenet{i}"), out=pres[i + 1])
        W0 = P["decoder/attention_lstm/kernel"]
        K.linear(pres[-1], W0[:pres[-1].shape[-1]], P["decoder/attention_lstm/bias"], out=X0)
    return {"xin": xin, "pres": pres, "X0": X0, "hist": None if hist is None else hist[1]}


def persistent_ineligible_reason(d: Dims, B: int, N: int, attn_tile: int = 32) -> Optional[str]:
    """Why sat_decoder_attention_fwd / sat_decoder_lstms_fwd (one launch for all T' steps) cannot
    take this shape, or None when they can (the self-attention-tacotron configs: one utterance
    per 8 workgroups for N <= 256, four per 32 otherwise, all of them resident on 256 CUs)."""
    if not (d.att1 == "forward" and d.att2 == "additive"):
        return f"attention kinds ({d.att1}, {d.att2}) are not (forward, additive)"
    if attn_tile != 32:
        return f"attn_tile {attn_tile} != 32"
    dims = (d.att_rnn, d.m1, d.m2, d.d1, d.d2, d.loc_f, d.loc_k, d.dec)
    if dims != (256, 256, 32, 224, 32, 5, 10, 256):
        return f"layer widths {dims} differ from the compiled (256, 256, 32, 224, 32, 5, 10, 256)"
    if not 0 < B <= 32:
        return f"per-GPU batch {B} outside 1..32"
    if ((B + 7) // 8) * ((N + 31) // 32) > 32:
        return (f"ceil(B/8) * ceil(N/32) = {((B + 7) // 8) * ((N + 31) // 32)} > 32 groups of "
                f"positions (B={B}, N={N}: more workgroups than CUs)")
    return None


def persistent_eligible(d: Dims, B: int, N: int, attn_tile: int = 32) -> bool:
    """Shapes sat_decoder_attention_fwd and sat_decoder_lstms_fwd are compiled for (the
    self-attention-tacotron configs)."""
    return persistent_ineligible_reason(d, B, N, attn_tile) is None


class PersistentFallbackWarning(RuntimeWarning):
    """A training / eval shape left the one-launch persistent decoder for the per-step launch
    path (several times slower per step; BASELINE.md section 3 lists the measured cost)."""


_FALLBACK_WARNED = set()


def use_persistent(d: Dims, B: int, N: int, attn_tile: int = 32, persistent: bool = True) -> bool:
    """The decoder path for this shape.  ``persistent=True`` (the engine default) takes the
    persistent kernels when eligible and otherwise WARNS once per (B, N) before falling back
    to the per-step launches; ``persistent=False`` asks for the per-step path silently."""
    if not persistent:
        return False
    why = persistent_ineligible_reason(d, B, N, attn_tile)
    if why is None:
        return True
    if (B, N, why) not in _FALLBACK_WARNED:
        _FALLBACK_WARNED.add((B, N, why))
        warnings.warn(f"decoder falls back to the per-step launch path: {why} "
                      f"(pass persistent_decoder=False to choose it explicitly)",
                      PersistentFallbackWarning, stacklevel=3)
    return False


def decoder_forward(P: Dict[str, torch.Tensor], hp, d: Dims, m1: torch.Tensor, m2: torch.Tensor,
                    lengths: torch.Tensor, targets: torch.Tensor,
                    masks: Optional[Dict[str, torch.Tensor]], attn_tile: int = 32,
                    spk: Optional[torch.Tensor] = None, pipe: Pipeline = SEQUENTIAL,
                    persistent: bool = False, scratch=None, keep_tanh: bool = True,
                    inputs: Optional[Dict[str, object]] = None):
    """Forward of the teacher-forced decoder; returns (D [T', B, dec], DecoderSaved).

    ``persistent`` runs the attention chain (attention RNN + query + dual-source attention) for
    all steps as ONE persistent launch (``sat_decoder_attention_fwd``) when the shapes allow,
    then the two decoder LSTMs as a two-problem wavefront; otherwise the per-step launches.
    ``keep_tanh`` keeps the energies' tanh for the persistent BPTT (off for inference).
    ``inputs``: the teacher frames, prenets and attention-RNN input projection already formed
    by ``decoder_inputs`` (model_forward runs them on a second stream beside the encoder)."""
    dev = m1.device
    B, N, _ = m1.shape
    r, nf = d.r, hp.n_feed_frame
    Tp = targets.shape[1] // r
    A, Dd = d.att_rnn, d.dec
    M1, M2, D1, D2 = d.m1, d.m2, d.d1, d.d2
    zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
    f32 = dict(device=dev, dtype=torch.float32)
    mk = (lambda name: masks[name]) if masks is not None else (lambda name: None)

    S = {}
    # ---- memories (TF _prepare_memory + memory_layer), once per utterance
    V1 = K.seq_mask(m1, lengths)
    V2 = K.seq_mask(m2, lengths)
    K1 = K.linear(V1, P["decoder/attention1/memory_layer/kernel"])
    K2 = K.linear(V2, P["decoder/attention2/memory_layer/kernel"])
    S.update(V1=V1, V2=V2, K1=K1, K2=K2)

    # ---- prenets over all frames (teacher forcing), dropout fused as a multiplicative epilogue
    xin = teacher_inputs(targets, r, nf) if inputs is None else inputs["xin"]
    pre = xin
    pres = [xin] if inputs is None else inputs["pres"]
    if inputs is not None:
        pre = pres[-1]
    elif spk is not None:
        # MultiSpeakerPreNet (modules/multi_speaker_modules.py:27-32): the speaker term is one
        # [B, p0] row per utterance, broadcast over the T' steps by a zero batch stride of the
        # step-major [T', B, .] GEMM's residual operand
        p0 = d.dec_prenet[0]
        ms = "decoder/prenet0"
        sp = K.linear(spk, P[f"{ms}/speaker_projection/kernel"],
                      P[f"{ms}/speaker_projection/bias"], act="softsign")          # [B, p0]
        y0 = K.linear(xin, P[f"{ms}/dense0/kernel"], P[f"{ms}/dense0/bias"], act="relu")
        d0 = K.gemm(xin, P[f"{ms}/dense0/kernel"], bias=P[f"{ms}/dense0/bias"], act="relu",
                    add=sp.unsqueeze(0).expand(Tp, B, p0))
        S["ms_prenet"] = dict(spk=spk, sp=sp, y0=y0)
        pres = [d0]
        pre = K.linear(d0, P[f"{ms}/dense/kernel"], P[f"{ms}/dense/bias"], act="relu",
                       mul=mk("dec/prenet0"))
        pres.append(pre)
    if inputs is None:
        for i in range(len(pres) - 1, len(d.dec_prenet)):
            pre = K.linear(pre, P[f"decoder/prenet{i}/kernel"], P[f"decoder/prenet{i}/bias"],
                           act="relu", mul=mk(f"dec/prenet{i}"))
            pres.append(pre)
    S["prenet"] = pres
    S["xin"] = xin
    p_w = pre.shape[-1]

    # ---- attention RNN (ZoneoutLSTM A) input projection of the prenet part
    W0 = P["decoder/attention_lstm/kernel"]          # [p + M1 + M2 + A, 4A] (gate-interleaved)
    X0 = (K.linear(pre, W0[:p_w], P["decoder/attention_lstm/bias"]) if inputs is None
          else inputs["X0"])                         # [T', B, 4A]
    R0 = M1 + M2 + A                                 # recurrent input [c1 | c2 | h0]
    # zero-initialised state histories (row 0 = initial state), one fill for all of them and
    # for the decoder LSTMs' c / h histories below
    hist = inputs.get("hist") if inputs is not None else None
    if hist is not None and tuple(hist[2].shape) == (Tp + 1, B, N):
        REC0, C0, S1, AL1, c1z, h1z, c2z, h2z = hist      # zeroed on the inputs' side stream
    else:
        REC0, C0, S1, AL1, c1z, h1z, c2z, h2z = K.zeros_group(*_state_shapes(d, Tp, B, N),
                                                              device=dev)
        AL1[0, :, 0] = 1.0                           # forward_attention.py:131-133
    H0RAW = torch.empty(Tp, B, A, **f32)
    G0 = torch.empty(Tp, B, 4 * A, **f32)
    Q = torch.empty(Tp, B, D1 + D2, **f32)
    S2 = torch.empty(Tp, B, N, **f32)
    ST = torch.empty(Tp, B, 4, **f32)
    # location features f_t of every step (forward attention): the backward's parameter-gradient
    # pass recomputes the energies from them
    LOC = torch.empty(Tp, B, N, max(d.loc_f, 1), **f32) if d.att1 == "forward" else None
    ntiles = (N + attn_tile - 1) // attn_tile
    pst = K.part_stride(M1, M2)
    E1 = torch.empty(B, N, **f32)
    E2 = torch.empty(B, N, **f32)
    PART = torch.empty(B, ntiles, pst, **f32)
    att1_fwd = 1 if d.att1 == "forward" else 0
    if d.att2 != "additive":
        raise NotImplementedError("attention2 must be 'additive' (hparams.py:98)")
    a1 = "decoder/attention1"
    Wr0 = W0[p_w:]
    # query layers of both mechanisms, transposed once per step so the per-decoder-step query
    # product is a skinny row-dot ([B, A] x [D1+D2, A]^T)
    # (made on first use: the persistent path reads the kernels directly)
    qt_box = []

    def query_t():
        if not qt_box:
            QT = torch.empty(D1 + D2, A, **f32)
            K.transpose(P[f"{a1}/query_layer/kernel"], QT[:D1])
            K.transpose(P["decoder/attention2/query_layer/kernel"], QT[D1:])
            qt_box.append(QT)
        return qt_box[0]
    zc0, zh0 = mk("dec/lstm0/zc"), mk("dec/lstm0/zh")

    def lstm0_desc(t):
        return dict(B=B, U=A, K=R0, t=t, xproj=X0[t], rin=REC0[t], W=Wr0, c_prev=C0[t],
                    h_prev=REC0[t, :, M1 + M2:], mask_c=None if zc0 is None else zc0[t],
                    mask_h=None if zh0 is None else zh0[t], zc=zc, zh=zh, h_raw=H0RAW[t],
                    c_out=C0[t + 1], h_out=REC0[t + 1, :, M1 + M2:], gates=G0[t])

    def attention_rest(t):
        K.rowdot(H0RAW[t], query_t(), Q[t])
        K.attn_step_fwd(
            B=B, N=N, D1=D1, M1=M1, D2=D2, M2=M2, F=d.loc_f, KW=d.loc_k, NT=attn_tile,
            ntiles=ntiles, att1_forward=att1_fwd, u=0.5, q=Q[t], q_sb=D1 + D2,
            K1=K1, V1=V1, K2=K2, V2=V2, lengths=lengths, s_prev=S1[t], a_prev=AL1[t],
            v1=P[f"{a1}/attention_variable"] if att1_fwd else P[f"{a1}/attention_v"],
            b1=P[f"{a1}/attention_bias"] if att1_fwd else None,
            convW=P[f"{a1}/location_conv/kernel"] if att1_fwd else None,
            convb=P[f"{a1}/location_conv/bias"] if att1_fwd else None,
            locW=P[f"{a1}/location_layer/kernel"] if att1_fwd else None,
            v2=P["decoder/attention2/attention_v"], e1=E1, e2=E2, part=PART, part_stride=pst,
            s_out=S1[t + 1], a_out=AL1[t + 1], s2_out=S2[t], ctx=REC0[t + 1], ctx_sb=R0,
            stats=ST[t], loc_out=None if LOC is None else LOC[t])

    # ---- decoder LSTM 1: input o_t = [h0'_t | c1_t | c2_t]  (ConcatOutputAndAttentionWrapper)
    W1 = P["decoder/lstm1/kernel"]                   # [A + M1 + M2 + D, 4D]
    W2 = P["decoder/lstm2/kernel"]                   # [D + D, 4D]
    X1 = torch.empty(Tp, B, 4 * Dd, **f32)
    X2 = torch.empty(Tp, B, 4 * Dd, **f32)
    L1 = _lstm_buffers(Tp, B, Dd, f32, c1z, h1z)
    L2 = _lstm_buffers(Tp, B, Dd, f32, c2z, h2z)
    m1c, m1h, m2c, m2h = (mk("dec/lstm1/zc"), mk("dec/lstm1/zh"), mk("dec/lstm2/zc"),
                          mk("dec/lstm2/zh"))

    def x1_chunk(a, b):
        n = (b - a) * B
        x1 = X1[a:b].view(n, 4 * Dd)
        # ONE reduction over [h0'_t | c1_t | c2_t]: the raw attention-RNN output and the contexts
        # (REC0 row t+1) are the two A segments of W1x
        K.gemm(H0RAW[a:b].reshape(n, A), W1[:A + M1 + M2], x1, bias=P["decoder/lstm1/bias"],
               A2=REC0[a + 1:b + 1].reshape(n, R0)[:, :M1 + M2])

    def x2_chunk(a, b):
        n = (b - a) * B
        K.linear(L1[0][a:b].reshape(n, Dd), W2[:Dd], P["decoder/lstm2/bias"],
                 out=X2[a:b].view(n, 4 * Dd))

    def lstm1_desc(t):
        return _lstm_desc(X1, W1[A + M1 + M2:], t, B, Dd, zc, zh, m1c, m1h, L1)

    def lstm2_desc(t):
        return _lstm_desc(X2, W2[Dd:], t, B, Dd, zc, zh, m2c, m2h, L2)

    if use_persistent(d, B, N, attn_tile, persistent):
        if scratch is None:
            scratch = K.DecoderAttentionScratch(B, N, dev)
        # tanh of every energy pre-activation, kept for the persistent BPTT ([T', B, N, D1+D2]:
        # 3.3 GB at the LJSpeech batch-32 bench shape -- HBM is 288 GB, transcendentals are not
        # cheap on the BPTT's critical path)
        ZH = torch.empty(Tp, B, N, D1 + D2, **f32) if keep_tanh else None
        S["ZH"] = ZH
        K.decoder_attention_fwd(
            B=B, N=N, T=Tp, U=A, M1=M1, M2=M2, D1=D1, D2=D2, F=d.loc_f, KW=d.loc_k, u=0.5,
            zc=zc, zh=zh, X0=X0, W0r=Wr0, Wq1=P[f"{a1}/query_layer/kernel"],
            Wq2=P["decoder/attention2/query_layer/kernel"], K1=K1, V1=V1, K2=K2, V2=V2,
            lengths=lengths, v1=P[f"{a1}/attention_variable"], b1=P[f"{a1}/attention_bias"],
            convW=P[f"{a1}/location_conv/kernel"], convb=P[f"{a1}/location_conv/bias"],
            locW=P[f"{a1}/location_layer/kernel"], v2=P["decoder/attention2/attention_v"],
            mask_c=zc0, mask_h=zh0, REC0=REC0, C0=C0, H0RAW=H0RAW, G0=G0, Q=Q, S1=S1, AL1=AL1,
            S2=S2, ST=ST, LOC=LOC, E=scratch.E, PART=scratch.PART, QP=scratch.QP, ctr=scratch.ctr,
            err=scratch.err, ZH=ZH)
        S["attn_scratch"] = scratch
        # decoder LSTMs: all of LSTM1's input projection at once, then both layers' recurrences
        # as ONE persistent launch (LSTM2 one step behind LSTM1, in-kernel group barriers);
        # LSTM2's input projection happens inside it, so X2 is never materialised
        x1_chunk(0, Tp)
        X2 = None
        K.decoder_lstms_fwd(
            B=B, T=Tp, U=Dd, zc=zc, zh=zh, X1=X1, W1r=W1[A + M1 + M2:], W2=W2,
            b2=P["decoder/lstm2/bias"], mask1_c=m1c, mask1_h=m1h, mask2_c=m2c, mask2_h=m2h,
            H1RAW=L1[0], C1S=L1[1], H1S=L1[2], G1=L1[3], H2RAW=L2[0], C2S=L2[1], H2S=L2[2],
            G2=L2[3], xch=scratch.lstm_xch, err=scratch.lstm_err[0])
    elif not pipe.enabled:          # layer by layer
        for t in range(Tp):
            K.lstm_step_fwd(**lstm0_desc(t))
            attention_rest(t)
        x1_chunk(0, Tp)
        for t in range(Tp):
            K.lstm_step_fwd(**lstm1_desc(t))
        x2_chunk(0, Tp)
        for t in range(Tp):
            K.lstm_step_fwd(**lstm2_desc(t))
    else:                         # wavefront: LSTM1 C steps and LSTM2 2C steps behind
        C = pipe.chunk
        x1_at = pipe.finishing(Tp, 0)
        x2_at = pipe.finishing(Tp, C)
        for i in range(Tp + 2 * C):
            steps = []
            if i < Tp:
                steps.append(lstm0_desc(i))
            if 0 <= i - C < Tp:
                steps.append(lstm1_desc(i - C))
            if 0 <= i - 2 * C < Tp:
                steps.append(lstm2_desc(i - 2 * C))
            if steps:
                K.lstm_steps_fwd(steps)
            if i < Tp:
                attention_rest(i)
            if i in x1_at:
                x1_chunk(*x1_at[i])
            if i in x2_at:
                x2_chunk(*x2_at[i])
    S.update(X0=X0, REC0=REC0, C0=C0, H0RAW=H0RAW, G0=G0, Q=Q, S1=S1, AL1=AL1, S2=S2, ST=ST,
             LOC=LOC)
    H1RAW, C1S, H1S, G1 = L1
    H2RAW, C2S, H2S, G2 = L2
    S.update(X1=X1, H1RAW=H1RAW, C1S=C1S, H1S=H1S, G1=G1, X2=X2, H2RAW=H2RAW, C2S=C2S,
             H2S=H2S, G2=G2)
    return H2RAW, DecoderSaved(B, N, Tp, S)


def _lstm_buffers(Tp, B, U, f32, c=None, h=None):
    """(h_raw [T',B,U], c [T'+1,B,U], h [T'+1,B,U], gates [T',B,4U]) histories (c, h zeroed:
    given from a zeros_group, or allocated here)."""
    return (torch.empty(Tp, B, U, **f32),
            c if c is not None else K.zeros(Tp + 1, B, U, device=f32["device"]),
            h if h is not None else K.zeros(Tp + 1, B, U, device=f32["device"]),
            torch.empty(Tp, B, 4 * U, **f32))


def _lstm_desc(X, Wr, t, B, U, zc, zh, mc, mh, bufs):
    HRAW, CS, HS, G = bufs
    return dict(B=B, U=U, K=U, t=t, xproj=X[t], rin=HS[t], W=Wr, c_prev=CS[t], h_prev=HS[t],
                mask_c=None if mc is None else mc[t], mask_h=None if mh is None else mh[t],
                zc=zc, zh=zh, h_raw=HRAW[t], c_out=CS[t + 1], h_out=HS[t + 1], gates=G[t])
