"""Free-running (PREDICT) decoding on libsat_hip -- BASELINE.json configs[4] (C5).

Mirrors the inference branch of ``RNNTransformer.__call__`` (modules/module.py:766-784):
``dynamic_decode`` over ``OutputAndStopTokenTransparentWrapper(TransformerWrapper(
RNNStateHistoryWrapper(DecoderRNNV2)))`` (modules/rnn_wrappers.py:47-124, 188-214) driven by the
tacotron2 ``StopTokenBasedInferenceHelper`` (analog modules/helpers.py:111-160):

* step 0 feeds the go frame (zeros), step t+1 the last predicted frame of step t
  (``mel_t[:, -num_mels * n_feed:]``);
* the decoder cell is the training one in eval mode (no prenet dropout --
  ``apply_dropout_on_inference=False``, hparams.py:105 -- zoneout blend);
* ``TransformerWrapper`` re-runs the causal self-attention over the whole state history every
  step and keeps the last row.  Causal attention makes row t independent of later rows, so the
  row equals one query against a key/value cache of the history (the equivalence
  modules/transformer_test.py:44-90 pins): here each step appends its key/value row to a
  device-resident cache ``[B, max_iters, width]`` and attends once -- O(T) per step, not O(T^2);
* ``is_finished``: after step t, ``t > min_iters`` and ``sigmoid(stop_t) > 0.5`` for every
  utterance; evaluated on the device (``sat_stop_check``) and read by the host once per chunk
  of steps, the outputs are then cut at the first finished step (the steps computed past it
  never feed anything the reference returns).

Forced-alignment mode (``forced_alignments=(A1, A2)``, the second decoder pass of model_fn
under ``use_forced_alignment_mode``, models/models.py:118-148): the mechanisms are
``TeacherForcing{Forward,Additive}Attention`` (modules/teacher_forcing_attention.py:13-78), so
step t's alignments are the given ``A[:, t]`` and the contexts are ``A[:, t] . values``; the
helper is ``OneHotValidationHelper(teacher_forcing=False)`` (modules/helpers.py:61-108): step
t+1 is fed the per-frame softmax over the feature bins of step t's output (``feed="softmax"``,
the fork's code-prediction feedback, :100-104) and the loop runs exactly T' = A.shape[1] steps
(``finished = time + 1 >= num_steps``, :101), with no stop-token termination.

Every arithmetic op is a libsat_hip kernel; torch allocates, views and copies.
"""

from __future__ import annotations

import math
from typing import Dict, Optional

import torch

from . import kernels as K
from .model import BNState, encoder_fwd
from .params import Dims


class FreeRunningDecoder:
    """One free-running decode of a batch (eval semantics).  ``check_every`` = decoder steps
    between host reads of the device-side finished flag."""

    def __init__(self, model, max_iters: Optional[int] = None, min_iters: int = 10,
                 check_every: int = 25, forced_alignments=None, feed: str = "mel"):
        self.m = model
        self.hp = model.hp
        self.d: Dims = model.d
        self.max_iters = int(self.hp.max_iters if max_iters is None else max_iters)
        self.min_iters = int(min_iters)
        self.check_every = max(1, int(check_every))
        if feed not in ("mel", "softmax"):
            raise ValueError(f"feed must be 'mel' or 'softmax', got {feed!r}")
        self.feed = feed
        self.forced = None
        if forced_alignments is not None:
            a1, a2 = forced_alignments
            if a1.shape != a2.shape or a1.dim() != 3:
                raise ValueError("forced alignments must be two [B, T', N] tensors")
            self.forced = (a1.contiguous(), a2.contiguous())
            self.max_iters = int(a1.shape[1])

    # ------------------------------------------------------------------ one decode
    @torch.no_grad()
    def run(self, batch: Dict[str, torch.Tensor]) -> Dict[str, object]:
        m, hp, d = self.m, self.hp, self.d
        P, dev = m.P, m.device
        ids, lengths = batch["source"], batch["source_length"]
        B, N = ids.shape
        sv = {}
        m1, m2 = encoder_fwd(P, m.bn, hp, d, ids, lengths, None, False, m.ws, sv)
        spk = None
        if d.multi_speaker:
            spk = torch.empty(B, d.spk_dim, device=dev)
            err = torch.zeros(1, dtype=torch.int32, device=dev)
            K.embedding_fwd(P["speaker_embedding"], batch["speaker_id"], spk, d.spk_offset, err)
        Tm = self.max_iters
        f32 = dict(device=dev, dtype=torch.float32)
        forced = self.forced
        if forced is not None and tuple(forced[0].shape) != (B, Tm, N):
            raise ValueError(f"forced alignments must be [B={B}, T', N={N}], got "
                             f"{tuple(forced[0].shape)}")
        M, r, nf = d.num_mels, d.r, hp.n_feed_frame
        A, Dd, M1, M2, D1, D2 = d.att_rnn, d.dec, d.m1, d.m2, d.d1, d.d2
        R0 = M1 + M2 + A
        zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
        a1, a2 = "decoder/attention1", "decoder/attention2"
        att1_fwd = 1 if d.att1 == "forward" else 0
        if d.att2 != "additive":
            raise NotImplementedError("attention2 must be 'additive' (hparams.py:98)")

        # ---- memories (TF _prepare_memory + memory_layer)
        V1 = K.seq_mask(m1, lengths)
        V2 = K.seq_mask(m2, lengths)
        K1 = K.linear(V1, P[f"{a1}/memory_layer/kernel"])
        K2 = K.linear(V2, P[f"{a2}/memory_layer/kernel"])
        # ---- state (step-major histories)
        MEL = torch.zeros(Tm, B, M * r, **f32)
        STOP = torch.zeros(Tm, B, 1, **f32)
        GO = torch.zeros(B, M * nf, **f32)
        SMX = torch.empty(B, M * r, **f32)                # softmax feedback (feed="softmax")
        REC0 = torch.zeros(Tm + 1, B, R0, **f32)          # [c1 | c2 | h0] per step
        C0 = torch.zeros(2, B, A, **f32)
        H0RAW = torch.empty(B, A, **f32)
        L1 = [torch.zeros(2, B, Dd, **f32), torch.zeros(2, B, Dd, **f32)]   # c, h ping-pong
        L2 = [torch.zeros(2, B, Dd, **f32), torch.zeros(2, B, Dd, **f32)]
        H1RAW = torch.empty(B, Dd, **f32)
        H2RAW = torch.empty(B, Dd, **f32)
        GA = torch.empty(B, 4 * A, **f32)                 # activated gates (unused at inference)
        GD = torch.empty(B, 4 * Dd, **f32)
        X0 = torch.empty(B, 4 * A, **f32)
        X1 = torch.empty(B, 4 * Dd, **f32)
        X2 = torch.empty(B, 4 * Dd, **f32)
        Q = torch.empty(B, D1 + D2, **f32)
        S1 = torch.zeros(Tm + 1, B, N, **f32)
        AL1 = torch.zeros(Tm + 1, B, N, **f32)
        AL1[0, :, 0] = 1.0                                # forward_attention.py:131-133
        S2 = torch.zeros(Tm, B, N, **f32)
        ntiles = (N + 31) // 32
        pst = K.part_stride(M1, M2)
        E1 = torch.empty(B, N, **f32)
        E2 = torch.empty(B, N, **f32)
        PART = torch.empty(B, ntiles, pst, **f32)
        QT = torch.empty(D1 + D2, A, **f32)
        K.transpose(P[f"{a1}/query_layer/kernel"], QT[:D1])
        K.transpose(P[f"{a2}/query_layer/kernel"], QT[D1:])
        W0 = P["decoder/attention_lstm/kernel"]
        W1 = P["decoder/lstm1/kernel"]
        W2 = P["decoder/lstm2/kernel"]
        p_w = d.dec_prenet[-1]
        # ---- decoder self-attention key/value caches, one per hop
        H, dsa = d.dec_heads, d.dsa
        dh = dsa // H
        KC = [torch.zeros(B, Tm, dsa, **f32) for _ in range(d.dec_hops)]
        VC = [torch.zeros(B, Tm, dsa, **f32) for _ in range(d.dec_hops)]
        # row t of each hop's causal probabilities (= the final step's full [T', T'] matrix)
        SA_P = [torch.zeros(B, H, Tm, Tm, **f32) for _ in range(d.dec_hops)]
        state = torch.full((1,), -1, dtype=torch.int32, device=dev)
        sp = None
        if spk is not None:
            ms = "decoder/prenet0"
            sp = K.linear(spk, P[f"{ms}/speaker_projection/kernel"],
                          P[f"{ms}/speaker_projection/bias"], act="softsign")

        def prenets(x):
            if sp is not None:                            # multi_speaker_modules.py:27-32
                ms = "decoder/prenet0"
                y = K.gemm(x, P[f"{ms}/dense0/kernel"], bias=P[f"{ms}/dense0/bias"], act="relu",
                           add=sp)
                y = K.linear(y, P[f"{ms}/dense/kernel"], P[f"{ms}/dense/bias"], act="relu")
                start = 1
            else:
                y, start = x, 0
            for i in range(start, len(d.dec_prenet)):
                y = K.linear(y, P[f"decoder/prenet{i}/kernel"], P[f"decoder/prenet{i}/bias"],
                             act="relu")
            return y

        def head_step(h, t):
            """TransformerWrapper row t + OutputAndStopTokenTransparentWrapper projections."""
            z = h
            for hop in range(d.dec_hops):
                sc = f"decoder/self_attention{hop}"
                mh = f"{sc}/mha"
                q = K.linear(z, P[f"{mh}/query_projection/kernel"], P[f"{mh}/query_projection/bias"])
                K.linear(z, P[f"{mh}/key_projection/kernel"], P[f"{mh}/key_projection/bias"],
                         out=KC[hop][:, t])
                K.linear(z, P[f"{mh}/value_projection/kernel"],
                         P[f"{mh}/value_projection/bias"], out=VC[hop][:, t])
                qh = q.view(B, 1, H, dh).permute(0, 2, 1, 3)              # [B, H, 1, dh]
                kh = KC[hop][:, :t + 1].view(B, t + 1, H, dh).permute(0, 2, 3, 1)
                vh = VC[hop][:, :t + 1].view(B, t + 1, H, dh).permute(0, 2, 1, 3)
                S = K.gemm(qh, kh)                                        # [B, H, 1, t+1]
                Pc = torch.empty_like(S)
                K.softmax_fwd(S, Pc, None, None, causal=False, scale=1.0 / math.sqrt(dh))
                SA_P[hop][:, :, t:t + 1, :t + 1].copy_(Pc)
                o = torch.empty(B, dsa, **f32)
                K.gemm(Pc, vh, o.view(B, 1, H, dh).permute(0, 2, 1, 3))
                y = K.linear(o, P[f"{mh}/output_projection/kernel"],
                             P[f"{mh}/output_projection/bias"])
                z = K.linear(y, P[f"{sc}/transform/kernel"], P[f"{sc}/transform/bias"],
                             act="tanh", add=z)                           # z + tanh(Dense(.))
            K.linear(z, P["decoder/out_projection/kernel"], P["decoder/out_projection/bias"],
                     out=MEL[t])
            K.linear(z, P["decoder/stop_token_projection/kernel"],
                     P["decoder/stop_token_projection/bias"], out=STOP[t])

        def step(t):
            cur, nxt = t % 2, (t + 1) % 2
            if t == 0:
                x = GO
            elif self.feed == "softmax":                  # OneHotValidationHelper :100-104
                K.softmax_fwd(MEL[t - 1].view(B * r, M), SMX.view(B * r, M), causal=False)
                x = SMX[:, M * (r - nf):]
            else:
                x = MEL[t - 1][:, M * (r - nf):]
            pre = prenets(x)
            K.linear(pre, W0[:p_w], P["decoder/attention_lstm/bias"], out=X0)
            K.lstm_step_fwd(B=B, U=A, K=R0, t=t, xproj=X0, rin=REC0[t], W=W0[p_w:],
                            c_prev=C0[cur], h_prev=REC0[t, :, M1 + M2:], mask_c=None,
                            mask_h=None, zc=zc, zh=zh, h_raw=H0RAW, c_out=C0[nxt],
                            h_out=REC0[t + 1, :, M1 + M2:], gates=GA)
            if forced is not None:
                forced_step(t)
            else:
                attention_step(t)
            # LSTM1 on o_t = [h0'_t | c1_t | c2_t] (ConcatOutputAndAttentionWrapper)
            lstm_stack(t, cur, nxt)
            head_step(H2RAW, t)
            if forced is None:
                K.stop_check(STOP[t], t, self.min_iters, state)

        def forced_step(t):
            """TeacherForcing*Attention: alignments = A[:, t]; contexts = A[:, t] . values."""
            a1t, a2t = forced[0][:, t], forced[1][:, t]
            AL1[t + 1].copy_(a1t)
            S2[t].copy_(a2t)
            K.gemm(a1t.unsqueeze(1), V1, REC0[t + 1][:, :M1].unsqueeze(1))
            K.gemm(a2t.unsqueeze(1), V2, REC0[t + 1][:, M1:M1 + M2].unsqueeze(1))

        def attention_step(t):
            K.rowdot(H0RAW, QT, Q)
            K.attn_step_fwd(
                B=B, N=N, D1=D1, M1=M1, D2=D2, M2=M2, F=d.loc_f, KW=d.loc_k, NT=32,
                ntiles=ntiles, att1_forward=att1_fwd, u=0.5, q=Q, q_sb=D1 + D2,
                K1=K1, V1=V1, K2=K2, V2=V2, lengths=lengths, s_prev=S1[t], a_prev=AL1[t],
                v1=P[f"{a1}/attention_variable"] if att1_fwd else P[f"{a1}/attention_v"],
                b1=P[f"{a1}/attention_bias"] if att1_fwd else None,
                convW=P[f"{a1}/location_conv/kernel"] if att1_fwd else None,
                convb=P[f"{a1}/location_conv/bias"] if att1_fwd else None,
                locW=P[f"{a1}/location_layer/kernel"] if att1_fwd else None,
                v2=P[f"{a2}/attention_v"], e1=E1, e2=E2, part=PART, part_stride=pst,
                s_out=S1[t + 1], a_out=AL1[t + 1], s2_out=S2[t], ctx=REC0[t + 1], ctx_sb=R0,
                stats=None, loc_out=None)

        def lstm_stack(t, cur, nxt):
            K.linear(H0RAW, W1[:A], P["decoder/lstm1/bias"], out=X1)
            K.gemm(REC0[t + 1][:, :M1 + M2], W1[A:A + M1 + M2], X1, beta=1.0)
            K.lstm_step_fwd(B=B, U=Dd, K=Dd, t=t, xproj=X1, rin=L1[1][cur],
                            W=W1[A + M1 + M2:], c_prev=L1[0][cur], h_prev=L1[1][cur],
                            mask_c=None, mask_h=None, zc=zc, zh=zh, h_raw=H1RAW,
                            c_out=L1[0][nxt], h_out=L1[1][nxt], gates=GD)
            K.linear(H1RAW, W2[:Dd], P["decoder/lstm2/bias"], out=X2)
            K.lstm_step_fwd(B=B, U=Dd, K=Dd, t=t, xproj=X2, rin=L2[1][cur], W=W2[Dd:],
                            c_prev=L2[0][cur], h_prev=L2[1][cur], mask_c=None, mask_h=None,
                            zc=zc, zh=zh, h_raw=H2RAW, c_out=L2[0][nxt], h_out=L2[1][nxt],
                            gates=GD)

        steps = Tm
        for t in range(Tm):
            step(t)
            if forced is not None:
                continue
            if (t + 1) % self.check_every == 0 or t + 1 == Tm:
                first = int(state.item())
                if first >= 0:
                    steps = first + 1
                    break
        B_, T_ = B, steps
        mel = MEL[:T_].permute(1, 0, 2).reshape(B_, T_ * r, M)
        stop = STOP[:T_, :, 0].transpose(0, 1).contiguous()
        return {"mel": mel, "stop": stop, "steps": T_,
                "alignment1": AL1[1:T_ + 1].permute(1, 2, 0).contiguous(),   # [B, N, T']
                "alignment2": S2[:T_].permute(1, 2, 0).contiguous(),
                "decoder_self_alignments": [SA_P[h][:, :, :T_, :T_] for h in range(d.dec_hops)],
                "encoder_self_alignments": [sv[f"enc_sa{h}"]["P"] for h in range(d.enc_hops)],
                "m1": m1, "m2": m2}
