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

Validation decoding (``helper="validation"``: ``OneHotValidationHelper``, modules/helpers.py:61-108,
built by ``RNNTransformer.__call__`` with ``is_validation=True``, modules/module.py:733-738):
exactly T' = T/r steps of the batch's targets (``finished = time + 1 >= num_steps``, :101), no
stop-token termination; step t+1 is fed either the per-frame softmax of step t's output
(``feed="softmax"``, teacher_forcing=False: model_fn EVAL's ``loss``/``code_loss``/``done_loss``,
models/models.py:86-97, 159-173) or the target frame ``targets[:, t, -M*n_feed:]``
(``feed="target"``, teacher_forcing=True: the incremental branch modules/transformer_test.py:44-90
compares with the training branch).

Schedule: every buffer of a decode lives in a per-shape plan (static addresses), so a decode of
``check_every`` steps can be captured once as a hipGraph (``graphs=True``) and replayed: the host
issues one graph launch per chunk instead of ~30 kernel launches per step.

Every arithmetic op is a libsat_hip kernel; torch allocates, views and copies.
"""

from __future__ import annotations

import math
import warnings
from typing import Dict, Optional

import torch

from . import _lib
from . import kernels as K
from .model import BNState, encoder_fwd
from .params import Dims


class _Plan:
    """Static buffers of one decode shape (B, N, T_max) plus the per-step launch closures."""


class FreeRunningDecoder:
    """Incremental decoding of a batch with eval semantics (no dropout, zoneout blend, BN moving
    statistics).

    ``helper``: ``"stop_token"`` (PREDICT, StopTokenBasedInferenceHelper: up to ``max_iters``
    steps, stops once every utterance's stop token fired after ``min_iters``) or
    ``"validation"`` (OneHotValidationHelper: exactly T' = batch["mel"].shape[1] / r steps).
    ``feed``: what step t+1 is fed -- ``"mel"`` (the last predicted frame), ``"softmax"`` (its
    per-frame softmax over the feature bins) or ``"target"`` (the target frame; validation only).
    ``forced_alignments=(A1, A2)`` replays given alignments (TeacherForcing*Attention) and
    implies the validation helper with T' = A1.shape[1].
    ``check_every`` = decoder steps between host reads of the device-side finished flag (and
    the steps per captured graph when ``graphs=True``).
    ``persistent``: run the whole decode as ONE launch (``sat_decode_persistent``) -- None picks
    it whenever the shape allows (mel feedback, no forced alignments, single speaker, the
    LJSpeech decoder dimensions, B <= 8, N <= 256, T' <= 512), True requires it, False keeps the
    per-step launches."""

    def __init__(self, model, max_iters: Optional[int] = None, min_iters: int = 10,
                 check_every: int = 25, forced_alignments=None, feed: str = "mel",
                 helper: Optional[str] = None, graphs: bool = False,
                 persistent: Optional[bool] = None):
        self.m = model
        self.hp = model.hp
        self.d: Dims = model.d
        if getattr(self.hp, "apply_dropout_on_inference", False):
            # PreNet(apply_dropout_on_inference=True) keeps prenet dropout at inference
            # (modules/module.py:1513-1517); this build decodes with eval semantics only
            raise NotImplementedError("apply_dropout_on_inference=True is not supported: "
                                      "decoding runs with eval semantics (no prenet dropout)")
        self.max_iters = int(self.hp.max_iters if max_iters is None else max_iters)
        self.min_iters = int(min_iters)
        self.check_every = max(1, int(check_every))
        if feed not in ("mel", "softmax", "target"):
            raise ValueError(f"feed must be 'mel', 'softmax' or 'target', got {feed!r}")
        self.forced = None
        if forced_alignments is not None:
            a1, a2 = forced_alignments
            if a1.shape != a2.shape or a1.dim() != 3:
                raise ValueError("forced alignments must be two [B, T', N] tensors")
            self.forced = (a1.contiguous(), a2.contiguous())
            self.max_iters = int(a1.shape[1])
            helper = "validation" if helper is None else helper
        helper = "stop_token" if helper is None else helper
        if helper not in ("stop_token", "validation"):
            raise ValueError(f"helper must be 'stop_token' or 'validation', got {helper!r}")
        if feed == "target" and helper != "validation":
            raise ValueError("feed='target' (teacher forcing) needs the validation helper")
        if self.forced is not None and helper != "validation":
            raise ValueError("forced alignments run under the validation helper")
        self.helper = helper
        self.feed = feed
        self.graphs = bool(graphs)
        self.persistent = persistent
        self.last_path = None
        self._plans: Dict[tuple, _Plan] = {}

    # ------------------------------------------------------------------ plan (static buffers)
    def _plan(self, B: int, N: int, Tm: int) -> _Plan:
        key = (B, N, Tm)
        pl = self._plans.get(key)
        if pl is None:
            pl = self._build(B, N, Tm)
            use = self._persistent_ok(B, N, Tm)
            if self.persistent and not use:
                raise ValueError("persistent=True: this decode is not eligible for "
                                 "sat_decode_persistent (" + self._why_not(B, N, Tm) + ")")
            if use and self.persistent is not False:
                self._build_persistent(pl)
            self._plans[key] = pl
        return pl

    # ------------------------------------------------------------------ one-launch decode
    def _why_not(self, B: int, N: int, Tm: int) -> str:
        d, hp = self.d, self.hp
        dims = dict(dec_prenet=(256, 128), feed=80, att_rnn=256, m1=256, m2=32, d1=224, d2=32,
                    loc_k=10, loc_f=5, dec=256, dsa=256, dec_heads=2, dec_hops=1, num_mels=80, r=2,
                    att1="forward", att2="additive", multi_speaker=False)
        for k, v in dims.items():
            if getattr(d, k) != v:
                return f"{k}={getattr(d, k)!r}, needs {v!r}"
        if hp.n_feed_frame != 1:
            return "n_feed_frame != 1"
        if self.forced is not None or self.feed != "mel":
            return "forced alignments / non-mel feedback"
        if not (1 <= B <= 8 and 1 <= N <= 256 and 1 <= Tm <= 512):
            return f"B={B} (<= 8), N={N} (<= 256), T'={Tm} (<= 512)"
        if self.m.device.type != "cuda":
            return "not a GPU model"
        return ""

    def _persistent_ok(self, B: int, N: int, Tm: int) -> bool:
        return self._why_not(B, N, Tm) == ""

    def _build_persistent(self, pl: _Plan) -> None:
        """Packed weights of sat_decode_persistent (refilled from the parameters every run) and
        its scratch; see include/sat_abi.h SatDecodePersistent."""
        dev = self.m.device
        f32 = dict(device=dev, dtype=torch.float32)
        pl.pk = dict(Wzp=torch.empty(256, 256, **f32), bzp=torch.empty(1, 256, **f32),
                     Wq=torch.empty(256, 256, **f32), Wqku=torch.empty(256, 1024, **f32),
                     bqku=torch.zeros(1024, **f32), bz=torch.empty(1, 256, **f32),
                     tmp=torch.empty(2, 128, 256, **f32), y=torch.empty(1, 256, **f32))
        pl.scratch = torch.empty(K.decode_persistent_scratch_bytes(), dtype=torch.uint8,
                                 device=dev)
        pl.err = torch.zeros(1, dtype=torch.int32, device=dev)

    def _pack_persistent(self, pl: _Plan) -> None:
        """Fold the fed frame into the first prenet layer and the value / output projection /
        transform products into the cached rows (exact algebra, fp32 products):
        Wzp = W_out[:, fed] W_p0, bzp = b_out[fed] W_p0 + b_p0;
        Wqku = [W_q | W_k | W_v,h (W_o,h W_t)], bz = (b_v W_o + b_o) W_t + b_t."""
        P, d, pk = self.m.P, self.d, pl.pk
        M, r = d.num_mels, d.r
        fed = slice(M * (r - self.hp.n_feed_frame), M * r)
        Wp0 = P["decoder/prenet0/kernel"]
        K.gemm(pl.Wms[:, fed], Wp0, pk["Wzp"])
        K.gemm(pl.bms[fed].unsqueeze(0), Wp0, pk["bzp"], bias=P["decoder/prenet0/bias"])
        pk["Wq"][:, :d.d1].copy_(P["decoder/attention1/query_layer/kernel"])
        pk["Wq"][:, d.d1:].copy_(P["decoder/attention2/query_layer/kernel"])
        mh, sc = "decoder/self_attention0/mha", "decoder/self_attention0"
        dsa, dh = d.dsa, d.dsa // d.dec_heads
        Wqku = pk["Wqku"]
        Wqku[:, :dsa].copy_(P[f"{mh}/query_projection/kernel"])
        Wqku[:, dsa:2 * dsa].copy_(P[f"{mh}/key_projection/kernel"])
        pk["bqku"][:dsa].copy_(P[f"{mh}/query_projection/bias"])
        pk["bqku"][dsa:2 * dsa].copy_(P[f"{mh}/key_projection/bias"])
        Wv, Wo, Wt = (P[f"{mh}/value_projection/kernel"], P[f"{mh}/output_projection/kernel"],
                      P[f"{sc}/transform/kernel"])
        for h in range(d.dec_heads):
            K.gemm(Wo[h * dh:(h + 1) * dh], Wt, pk["tmp"][h])
            K.gemm(Wv[:, h * dh:(h + 1) * dh], pk["tmp"][h],
                   Wqku[:, 2 * dsa + h * dsa:3 * dsa + h * dsa])
        K.gemm(P[f"{mh}/value_projection/bias"].unsqueeze(0), Wo, pk["y"],
               bias=P[f"{mh}/output_projection/bias"])
        K.gemm(pk["y"], Wt, pk["bz"], bias=P[f"{sc}/transform/bias"])

    def _run_persistent(self, pl: _Plan, Tm: int) -> None:
        P, d, hp = self.m.P, self.d, self.hp
        a1, a2 = "decoder/attention1", "decoder/attention2"
        self._pack_persistent(pl)
        pk = pl.pk
        K.decode_persistent(
            B=pl.B, N=pl.N, T=Tm, min_iters=self.min_iters,
            stop_mode=1 if self.helper == "stop_token" else 0,
            zc=hp.zoneout_factor_cell, zh=hp.zoneout_factor_output, u=0.5,
            scale=1.0 / math.sqrt(d.dsa // d.dec_heads),
            lengths=pl.lengths, K1=pl.K1, V1=pl.V1, K2=pl.K2, V2=pl.V2,
            Wzp=pk["Wzp"], bzp=pk["bzp"], bp0=P["decoder/prenet0/bias"],
            Wp1=P["decoder/prenet1/kernel"], bp1=P["decoder/prenet1/bias"],
            W0=P["decoder/attention_lstm/kernel"], b0=P["decoder/attention_lstm/bias"],
            Wq=pk["Wq"], b1=P[f"{a1}/attention_bias"], v1=P[f"{a1}/attention_variable"],
            convW=P[f"{a1}/location_conv/kernel"], convb=P[f"{a1}/location_conv/bias"],
            locW=P[f"{a1}/location_layer/kernel"], v2=P[f"{a2}/attention_v"],
            W1=P["decoder/lstm1/kernel"], bl1=P["decoder/lstm1/bias"],
            W2=P["decoder/lstm2/kernel"], bl2=P["decoder/lstm2/bias"],
            Wqku=pk["Wqku"], bqku=pk["bqku"], bz=pk["bz"], Wms=pl.Wms, bms=pl.bms,
            MS=pl.MS, AL1=pl.AL1, S2=pl.S2, SA_P=pl.SA_P[0], state=pl.state,
            scratch=pl.scratch, scratch_bytes=pl.scratch.numel(), err=pl.err)

    def _try_persistent(self, pl: _Plan, Tm: int) -> Optional[str]:
        """Run the one-launch decode; None when it ran to the end, else why it did not (the
        library refused the launch, e.g. SAT_ERR_UNSUPPORTED on a device with fewer than 256
        co-resident workgroups, or a hand-off timed out and raised the error word)."""
        try:
            self._run_persistent(pl, Tm)
        except _lib.SatLibraryError as e:
            if e.rc != _lib.SAT_ERR_UNSUPPORTED:
                raise
            return str(e)
        if int(pl.err.item()) != 0:
            # not a refusal: the kernel started and a hand-off spin gave up -- a hang or a
            # regression in the one-launch decode, never silently replaced
            raise _lib.SatLibraryError("sat_decode_persistent: a hand-off timed out (error word "
                                       f"{int(pl.err.item())}); the grid was not co-resident "
                                       "or the kernel regressed")
        return None

    def _build(self, B: int, N: int, Tm: int) -> _Plan:
        m, hp, d = self.m, self.hp, self.d
        P, dev = m.P, m.device
        f32 = dict(device=dev, dtype=torch.float32)
        M, r, nf = d.num_mels, d.r, hp.n_feed_frame
        A, Dd, M1, M2, D1, D2 = d.att_rnn, d.dec, d.m1, d.m2, d.d1, d.d2
        R0 = M1 + M2 + A
        zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
        a1, a2 = "decoder/attention1", "decoder/attention2"
        att1_fwd = 1 if d.att1 == "forward" else 0
        if d.att2 != "additive":
            raise NotImplementedError("attention2 must be 'additive' (hparams.py:98)")
        pl = _Plan()
        pl.B, pl.N, pl.Tm = B, N, Tm
        # ---- inputs (copied in per run) and memories
        pl.lengths = torch.zeros(B, dtype=torch.int64, device=dev)
        pl.V1 = torch.zeros(B, N, M1, **f32)
        pl.V2 = torch.zeros(B, N, M2, **f32)
        pl.K1 = torch.zeros(B, N, D1, **f32)
        pl.K2 = torch.zeros(B, N, D2, **f32)
        pl.sp = torch.zeros(B, d.dec_prenet[0], **f32) if d.multi_speaker else None
        pl.XT = torch.zeros(Tm, B, M * nf, **f32) if self.feed == "target" else None
        pl.FA = ((torch.zeros(B, Tm, N, **f32), torch.zeros(B, Tm, N, **f32))
                 if self.forced is not None else None)
        # ---- state (step-major histories)
        W0 = P["decoder/attention_lstm/kernel"]
        W1 = P["decoder/lstm1/kernel"]
        W2 = P["decoder/lstm2/kernel"]
        p_w = d.dec_prenet[-1]
        # mel frame and stop logit of a step share one row [mel (M r) | stop | pad] written by ONE
        # product with the packed [W_mel | w_stop | 0] (rows 16-byte aligned)
        MSW = (M * r + 1 + 3) // 4 * 4
        pl.MS = MS = torch.zeros(Tm, B, MSW, **f32)
        pl.MEL = MEL = MS[..., :M * r]
        pl.STOP = STOP = MS[..., M * r:M * r + 1]
        pl.Wms = torch.zeros(d.dsa, MSW, **f32)
        pl.bms = torch.zeros(MSW, **f32)
        GO = torch.zeros(B, M * nf, **f32)
        SMX = torch.empty(B, M * r, **f32)                 # softmax feedback (feed="softmax")
        MELC = torch.empty(B, M * r, **f32)                 # contiguous copy for that feedback
        # the attention RNN's whole input row per step: [prenet out (p_w) | c1 | c2 | h0], so its
        # product (input projection included) is ONE step launch against the full kernel W0
        RX = p_w + R0
        pl.REC0X = REC0X = torch.zeros(Tm + 1, B, RX, **f32)
        pl.REC0 = REC0 = REC0X[..., p_w:]                  # [c1 | c2 | h0] per step (view)
        C0 = torch.zeros(2, B, A, **f32)
        H0RAW = torch.empty(B, A, **f32)
        L1 = [torch.zeros(2, B, Dd, **f32), torch.zeros(2, B, Dd, **f32)]   # c, h ping-pong
        L2 = [torch.zeros(2, B, Dd, **f32), torch.zeros(2, B, Dd, **f32)]
        H1RAW = torch.empty(B, Dd, **f32)
        H2RAW = torch.empty(B, Dd, **f32)
        GA = torch.empty(B, 4 * A, **f32)                  # activated gates (unused here)
        GD = torch.empty(B, 4 * Dd, **f32)
        Q = torch.empty(B, D1 + D2, **f32)
        pl.S1 = S1 = torch.zeros(Tm + 1, B, N, **f32)
        pl.AL1 = AL1 = torch.zeros(Tm + 1, B, N, **f32)
        pl.S2 = S2 = torch.zeros(Tm, B, N, **f32)
        ntiles = (N + 31) // 32
        pst = K.part_stride(M1, M2)
        E1 = torch.empty(B, N, **f32)
        E2 = torch.empty(B, N, **f32)
        PART = torch.empty(B, ntiles, pst, **f32)
        pl.QT = QT = torch.empty(D1 + D2, A, **f32)
        # ---- decoder self-attention: per hop one cache of [q | k | v] rows per step (the
        # q/k/v projections of a step are ONE product with the packed [Wq | Wk | Wv]), the
        # packed weights refreshed from the parameters at every run
        H, dsa = d.dec_heads, d.dsa
        dh = dsa // H
        pl.QKVC = QKVC = [torch.zeros(B, Tm, 3 * dsa, **f32) for _ in range(d.dec_hops)]
        pl.Wqkv = [torch.empty(dsa, 3 * dsa, **f32) for _ in range(d.dec_hops)]
        pl.bqkv = [torch.empty(3 * dsa, **f32) for _ in range(d.dec_hops)]
        OH = torch.empty(B, dsa, **f32)
        # row t of each hop's causal probabilities (= the final step's full [T', T'] matrix)
        pl.SA_P = SA_P = [torch.zeros(B, H, Tm, Tm, **f32) for _ in range(d.dec_hops)]
        pl.state = state = torch.full((1,), -1, dtype=torch.int32, device=dev)
        pl.zero_each_run = [REC0X, C0, L1[0], L1[1], L2[0], L2[1], S1, AL1, S2, MS]
        pl.graphs = {}
        lengths, V1, V2, K1, K2 = pl.lengths, pl.V1, pl.V2, pl.K1, pl.K2
        sp, XT, FA = pl.sp, pl.XT, pl.FA
        feed, forced_mode, stop_mode = self.feed, FA is not None, self.helper == "stop_token"
        min_iters = self.min_iters
        Wqkv, bqkv = pl.Wqkv, pl.bqkv
        Wms, bms = pl.Wms, pl.bms

        def prenets(x, out):
            """the decoder prenets on the fed frame; the last layer writes `out`"""
            L = len(d.dec_prenet)
            if sp is not None:                             # multi_speaker_modules.py:27-32
                ms = "decoder/prenet0"
                y = K.gemm(x, P[f"{ms}/dense0/kernel"], bias=P[f"{ms}/dense0/bias"], act="relu",
                           add=sp)
                y = K.linear(y, P[f"{ms}/dense/kernel"], P[f"{ms}/dense/bias"], act="relu",
                             out=out if L == 1 else None)
                start = 1
            else:
                y, start = x, 0
            for i in range(start, L):
                y = K.linear(y, P[f"decoder/prenet{i}/kernel"], P[f"decoder/prenet{i}/bias"],
                             act="relu", out=out if i == L - 1 else None)

        def head_step(h, t):
            """TransformerWrapper row t + OutputAndStopTokenTransparentWrapper projections:
            the packed q/k/v product writes cache row t, one fused launch attends over rows
            0..t (sat_decode_attention_step), then the output projection, the transform, and
            one product for the mel frame and the stop logit."""
            z = h
            for hop in range(d.dec_hops):
                sc = f"decoder/self_attention{hop}"
                mh = f"{sc}/mha"
                K.linear(z, Wqkv[hop], bqkv[hop], out=QKVC[hop][:, t])
                K.decode_attention_step(QKVC[hop], t, H, dsa, 1.0 / math.sqrt(dh), SA_P[hop],
                                        OH)
                y = K.linear(OH, P[f"{mh}/output_projection/kernel"],
                             P[f"{mh}/output_projection/bias"])
                z = K.linear(y, P[f"{sc}/transform/kernel"], P[f"{sc}/transform/bias"],
                             act="tanh", add=z)                           # z + tanh(Dense(.))
            K.linear(z, Wms, bms, out=MS[t])

        def forced_step(t):
            """TeacherForcing*Attention: alignments = A[:, t]; contexts = A[:, t] . values."""
            a1t, a2t = FA[0][:, t], FA[1][:, t]
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
                s_out=S1[t + 1], a_out=AL1[t + 1], s2_out=S2[t], ctx=REC0[t + 1], ctx_sb=RX,
                stats=None, loc_out=None)

        def lstm_stack(t, cur, nxt):
            # LSTM1 on [h0'_t | c1_t c2_t | h1_{t-1}] and LSTM2 on [h1'_t | h2_{t-1}], each one
            # step launch with its whole kernel (input projection included) and bias
            K.lstm_step_fwd(B=B, U=Dd, K=A + M1 + M2 + Dd, t=t, xproj=None,
                            bias=P["decoder/lstm1/bias"], rin=H0RAW,
                            rin1=REC0[t + 1][:, :M1 + M2], rin2=L1[1][cur], W=W1,
                            c_prev=L1[0][cur], h_prev=L1[1][cur], mask_c=None, mask_h=None,
                            zc=zc, zh=zh, h_raw=H1RAW, c_out=L1[0][nxt], h_out=L1[1][nxt],
                            gates=GD)
            K.lstm_step_fwd(B=B, U=Dd, K=Dd + Dd, t=t, xproj=None, bias=P["decoder/lstm2/bias"],
                            rin=H1RAW, rin1=L2[1][cur], W=W2, c_prev=L2[0][cur],
                            h_prev=L2[1][cur], mask_c=None, mask_h=None, zc=zc, zh=zh,
                            h_raw=H2RAW, c_out=L2[0][nxt], h_out=L2[1][nxt], gates=GD)

        def step(t):
            cur, nxt = t % 2, (t + 1) % 2
            if t == 0:
                x = GO
            elif feed == "target":                         # OneHotValidationHelper :103
                x = XT[t]
            elif feed == "softmax":                        # OneHotValidationHelper :100-104
                MELC.copy_(MEL[t - 1])
                K.softmax_fwd(MELC.view(B * r, M), SMX.view(B * r, M), causal=False)
                x = SMX[:, M * (r - nf):]
            else:
                x = MEL[t - 1][:, M * (r - nf):]
            prenets(x, REC0X[t][:, :p_w])
            # the attention RNN on [prenet | c1 c2 | h0_{t-1}] against its whole kernel
            K.lstm_step_fwd(B=B, U=A, K=RX, t=t, xproj=None,
                            bias=P["decoder/attention_lstm/bias"], rin=REC0X[t], W=W0,
                            c_prev=C0[cur], h_prev=REC0[t, :, M1 + M2:], mask_c=None,
                            mask_h=None, zc=zc, zh=zh, h_raw=H0RAW, c_out=C0[nxt],
                            h_out=REC0[t + 1, :, M1 + M2:], gates=GA)
            if forced_mode:
                forced_step(t)
            else:
                attention_step(t)
            # LSTM1 on o_t = [h0'_t | c1_t | c2_t] (ConcatOutputAndAttentionWrapper)
            lstm_stack(t, cur, nxt)
            head_step(H2RAW, t)
            if stop_mode:
                K.stop_check(STOP[t], t, min_iters, state)

        pl.step = step
        return pl

    # ------------------------------------------------------------------ one decode
    def _prepare(self, pl: _Plan, batch, spk_rows):
        """Per-run inputs into the plan's static buffers: memories, feeds, reset state."""
        m, hp, d = self.m, self.hp, self.d
        P = m.P
        B, N, Tm = pl.B, pl.N, pl.Tm
        for t in pl.zero_each_run:
            t.zero_()
        pl.AL1[0, :, 0] = 1.0                                 # forward_attention.py:131-133
        pl.state.fill_(-1)
        pl.lengths.copy_(batch["source_length"])
        K.transpose(P["decoder/attention1/query_layer/kernel"], pl.QT[:d.d1])
        K.transpose(P["decoder/attention2/query_layer/kernel"], pl.QT[d.d1:])
        dsa = d.dsa
        for hop in range(d.dec_hops):
            mh = f"decoder/self_attention{hop}/mha"
            for i, nm in enumerate(("query", "key", "value")):
                pl.Wqkv[hop][:, i * dsa:(i + 1) * dsa].copy_(P[f"{mh}/{nm}_projection/kernel"])
                pl.bqkv[hop][i * dsa:(i + 1) * dsa].copy_(P[f"{mh}/{nm}_projection/bias"])
        Mr = d.num_mels * d.r
        pl.Wms[:, :Mr].copy_(P["decoder/out_projection/kernel"])
        pl.Wms[:, Mr:Mr + 1].copy_(P["decoder/stop_token_projection/kernel"])
        pl.bms[:Mr].copy_(P["decoder/out_projection/bias"])
        pl.bms[Mr:Mr + 1].copy_(P["decoder/stop_token_projection/bias"])
        if pl.sp is not None:
            ms = "decoder/prenet0"
            K.linear(spk_rows, P[f"{ms}/speaker_projection/kernel"],
                     P[f"{ms}/speaker_projection/bias"], act="softsign", out=pl.sp)
        if pl.XT is not None:                                  # OneHotValidationHelper :103
            M, r, nf = d.num_mels, d.r, hp.n_feed_frame
            tg = batch["mel"].reshape(B, Tm, M * r)
            pl.XT[1:].copy_(tg[:, :-1, M * (r - nf):].transpose(0, 1))
        if pl.FA is not None:
            pl.FA[0].copy_(self.forced[0])
            pl.FA[1].copy_(self.forced[1])

    def _steps(self, pl: _Plan, a: int, b: int):
        if not self.graphs:
            for t in range(a, b):
                pl.step(t)
            return
        g = pl.graphs.get(a)
        if g is None:
            # capture on the plan's ONE side stream (the current stream's pending work is
            # joined first); the graph's private pool keeps every per-step temporary alive
            # across replays.  One stream per plan: the GEMM split-K workspace is keyed by
            # stream, so a fresh stream per chunk would allocate (and pin) a new workspace
            # inside every chunk's pool; the plan's stream gets its workspace before the first
            # capture, outside any pool.
            s = getattr(pl, "capture_stream", None)
            if s is None:
                s = pl.capture_stream = torch.cuda.Stream(device=self.m.device)
                with torch.cuda.stream(s):
                    K._gemm_ws(self.m.device)
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    for t in range(a, b):
                        pl.step(t)
            torch.cuda.current_stream().wait_stream(s)
            pl.graphs[a] = g
        g.replay()

    @torch.no_grad()
    def run(self, batch: Dict[str, torch.Tensor]) -> Dict[str, object]:
        m, hp, d = self.m, self.hp, self.d
        P, dev = m.P, m.device
        ids, lengths = batch["source"], batch["source_length"]
        B, N = ids.shape
        if self.helper == "validation" and self.forced is None:
            if "mel" not in batch:
                raise ValueError("the validation helper needs the batch's targets (batch['mel'])")
            Tm = int(batch["mel"].shape[1]) // d.r              # OneHotValidationHelper :69
        else:
            Tm = self.max_iters
        if self.forced is not None and tuple(self.forced[0].shape) != (B, Tm, N):
            raise ValueError(f"forced alignments must be [B={B}, T', N={N}], got "
                             f"{tuple(self.forced[0].shape)}")
        pl = self._plan(B, N, Tm)
        sv = {"keep_probs": True}      # the encoder self-alignments are an output here
        # the encoder BiLSTM as one launch (encoder_lstm.hip) like the training step's
        m1, m2 = encoder_fwd(P, m.bn, hp, d, ids, lengths, None, False, m.ws, sv,
                             persistent=m.persistent_decoder)
        spk = None
        if d.multi_speaker:
            spk = torch.empty(B, d.spk_dim, device=dev)
            err = torch.zeros(1, dtype=torch.int32, device=dev)
            K.embedding_fwd(P["speaker_embedding"], batch["speaker_id"], spk, d.spk_offset, err)
        def prepare():
            # ---- memories (TF _prepare_memory + memory_layer) into the plan's buffers
            self._prepare(pl, batch, spk)
            K.seq_mask(m1, pl.lengths, out=pl.V1)
            K.seq_mask(m2, pl.lengths, out=pl.V2)
            K.linear(pl.V1, P["decoder/attention1/memory_layer/kernel"], out=pl.K1)
            K.linear(pl.V2, P["decoder/attention2/memory_layer/kernel"], out=pl.K2)

        prepare()
        stop_mode = self.helper == "stop_token"
        steps = Tm
        self.last_path = "launches"
        if getattr(pl, "pk", None) is not None:
            why = self._try_persistent(pl, Tm)
            if why is None:
                self.last_path = "persistent"
                first = int(pl.state.item()) if stop_mode else -1
                if first >= 0:
                    steps = first + 1
            elif self.persistent:
                raise _lib.SatLibraryError("sat_decode_persistent: " + why)
            else:
                # persistent=None: the library refused the one-launch decode here
                # (SAT_ERR_UNSUPPORTED: too few co-resident workgroups on this device) -- this
                # plan decodes with the per-step launches from now on, starting again from
                # clean buffers, and says so
                warnings.warn("free-running decode falls back to per-step launches: " + why,
                              RuntimeWarning, stacklevel=2)
                pl.pk = None
                pl.err.zero_()
                prepare()
        for a in range(0, Tm if self.last_path == "launches" else 0, self.check_every):
            b = min(Tm, a + self.check_every)
            self._steps(pl, a, b)
            if stop_mode:
                first = int(pl.state.item())
                if first >= 0:
                    steps = first + 1
                    break
        T_ = steps
        r, M = d.r, d.num_mels
        # copies, never views of the plan's buffers: the next run() on this shape zeroes and
        # rewrites them (with B == 1 reshape / contiguous would return views)
        mel = pl.MEL[:T_].permute(1, 0, 2).reshape(B, T_ * r, M).clone()
        stop = pl.STOP[:T_, :, 0].transpose(0, 1).clone()
        return {"mel": mel, "stop": stop, "steps": T_,
                "alignment1": pl.AL1[1:T_ + 1].permute(1, 2, 0).clone(   # [B, N, T']
                    memory_format=torch.contiguous_format),
                "alignment2": pl.S2[:T_].permute(1, 2, 0).clone(memory_format=torch.contiguous_format),
                "decoder_self_alignments": [pl.SA_P[h][:, :, :T_, :T_].clone()
                                            for h in range(d.dec_hops)],
                "encoder_self_alignments": [sv[f"enc_sa{h}"]["P"] for h in range(d.enc_hops)],
                "m1": m1, "m2": m2}
