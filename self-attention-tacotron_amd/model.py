"""Self-attention Tacotron teacher-forced step on libsat_hip: encoder, self-attention heads, loss.

Forward mirrors ``model_fn`` TRAIN / EVAL-with-teacher (models/models.py:23-173):
  Embedding -> SelfAttentionCBHGEncoder (modules/module.py:425-438)
            -> DualSourceTransformerDecoder (decoder.py) -> RNNTransformer head (module.py:754-764)
            -> 0.1 * L1 + BCE loss.
Every arithmetic op is a libsat_hip kernel; torch only allocates, views and copies.
Activations that the backward needs are kept in ``Saved`` (HBM is 288 GB: store, don't recompute,
except the attention energies which the backward recomputes to avoid a [T', B, N, 224] tensor).
"""

from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import kernels as K
from . import params as PR
from .decoder import decoder_forward, decoder_inputs


class BNState:
    """Moving statistics of every BatchNormalization, two flat buffers (means, variances) laid
    out in ``params.bn_buffer_names`` order, so the 16 conv-bank BNs are one contiguous span."""

    def __init__(self, hp, device, storage: Optional[torch.Tensor] = None):
        """``storage``: an optional flat float view of ``numel(hp)`` elements to live in (the
        engine's data-parallel exchange arena, so the statistics ride in the gradient
        all-reduce)."""
        self.names = PR.bn_buffer_names(hp)
        self.offsets = {}
        off = 0
        for scope, ch in self.names:
            self.offsets[scope] = (off, ch)
            off += ch
        # one flat buffer [means | variances]: data-parallel replicas average it in ONE
        # collective (dp.exchange)
        init = torch.cat([torch.zeros(off), torch.ones(off)])
        if storage is None:
            self.buf = init.to(device)
        else:
            assert storage.numel() == init.numel(), "BN storage size"
            self.buf = storage
            self.buf.copy_(init)
        self.mean = self.buf[:off]
        self.var = self.buf[off:]

    @staticmethod
    def numel(hp) -> int:
        return 2 * sum(ch for _, ch in PR.bn_buffer_names(hp))

    def span(self, first_scope: str, count_ch: int):
        o, _ = self.offsets[first_scope]
        return self.mean[o:o + count_ch], self.var[o:o + count_ch]


def _contig_span(P: Dict[str, torch.Tensor], names: List[str]) -> torch.Tensor:
    """A view covering consecutive arena tensors (asserts adjacency)."""
    first = P[names[0]]
    n = sum(P[x].numel() for x in names)
    base = first.data_ptr()
    off = 0
    for x in names:
        if P[x].data_ptr() != base + 4 * off:
            raise RuntimeError(f"parameter {x} is not adjacent in the arena")
        off += P[x].numel()
    return first.view(-1).as_strided((n,), (1,))


def bank_fused(d, inp: torch.Tensor) -> bool:
    """The conv bank runs as ONE sat_cbhg_convbank launch per direction when its channel counts
    suit the LDS kernel (the configs' 128/128); otherwise one sat_gemm conv per kernel width."""
    return d.conv_ch % 64 == 0 and inp.shape[-1] % 64 == 0


def mha_fwd(x: torch.Tensor, P, scope: str, heads: int, causal: bool,
            probs_mask: Optional[torch.Tensor], sv: dict, key: str):
    """MultiHeadAttention (modules/self_attention.py:108-128) over x [B, L, W]: ONE
    sat_mha_fwd call (projections, per-head scores, masked softmax, contexts, output)."""
    B, L, W = x.shape
    model = P[f"{scope}/query_projection/kernel"].shape[1]
    out = P[f"{scope}/output_projection/kernel"].shape[1]
    dev = x.device
    qkv = torch.empty(3, B, L, model, device=dev)     # one buffer: a single batched Q/K/V product
    s = dict(x=x, q=qkv[0], k=qkv[1], v=qkv[2], o=torch.empty(B, L, model, device=dev),
             y=torch.empty(B, L, out, device=dev), mask=probs_mask, heads=heads,
             dh=model // heads, causal=causal, scope=scope)
    # the same rule as the library's flash_ok (csrc/mha.hip): 16-byte operands, the probability
    # mask included (a mask view at an unaligned arena offset takes the materialised path)
    aligned = all(t is None or t.data_ptr() % 16 == 0 for t in (probs_mask, *qkv))
    if aligned and K.flash_attn_ok(causal, model // heads, L) and not sv.get("keep_probs"):
        # the decoder head (causal, dh = 128) and the encoder's narrow heads: scores, softmax,
        # dropout and contexts fused per (utterance, head) -- only the row statistic is kept for
        # the backward (sv["keep_probs"]: the caller wants P itself, e.g. inference alignments)
        s["lse"] = torch.empty(B, heads, L, device=dev)
        s["P"] = s["Pd"] = None
    else:
        s["P"] = torch.empty(B, heads, L, L, device=dev)
        s["Pd"] = torch.empty_like(s["P"]) if probs_mask is not None else s["P"]
    d, _ = K.mha_desc(x, *(P[f"{scope}/{n}_projection/{t}"] for n in ("query", "key", "value",
                                                                        "output")
                           for t in ("kernel", "bias")), heads, causal, probs_mask, s)
    K.mha_fwd(d)
    sv[key] = s
    return s["y"]


def sa_transformer_fwd(x, P, scope, heads, causal, probs_mask, sv, key):
    """SelfAttentionTransformer.call (modules/module.py:363-371): x + tanh(Dense(MHA(x)))."""
    y = mha_fwd(x, P, f"{scope}/mha", heads, causal, probs_mask, sv, key)
    u = K.linear(y, P[f"{scope}/transform/kernel"], P[f"{scope}/transform/bias"], act="tanh")
    z = K.add(x, u)                                                  # residual (one launch)
    sv[key]["u"] = u
    sv[key]["z"] = z
    return z


def encoder_fwd(P, bn: BNState, hp, d: PR.Dims, ids, lengths, masks, training, ws, sv,
                persistent: bool = False, err: Optional[torch.Tensor] = None, before_lstm=None):
    """SelfAttentionCBHGEncoder.call (modules/module.py:425-438) -> (M1, M2).  ``err``: the
    int32 word the embedding's id-range check raises (zeroed here; default a fresh one).
    ``before_lstm``: called right before the BiLSTM launch (which holds only 2B CUs)."""
    dev = ids.device
    B, N = ids.shape
    mk = (lambda n: masks[n]) if masks is not None else (lambda n: None)
    emb = torch.empty(B, N, d.embed, device=dev)
    if err is None:
        err = K.zeros(1, dtype=torch.int32, device=dev)
    else:
        K.fill_(err)
    K.embedding_fwd(P["embedding"], ids, emb, 0, err)
    sv["emb_err"] = err
    x = emb
    pre = [emb]
    for i in range(len(d.enc_prenet)):                                # ext PreNet x2
        x = K.linear(x, P[f"encoder/prenet{i}/kernel"], P[f"encoder/prenet{i}/bias"], act="relu",
                     mul=mk(f"enc/prenet{i}"))
        pre.append(x)
    sv["enc_pre"] = pre
    inp = x
    C = d.conv_ch
    KC = d.max_k * C
    bank_pre = torch.empty(B, N, KC, device=dev)
    names = [f"encoder/cbhg/conv_bank/K{k}" for k in range(1, d.max_k + 1)]
    if bank_fused(d, inp):                                            # module.py:78
        K.conv_bank(inp, _contig_span(P, [f"{n}/kernel" for n in names]),
                    _contig_span(P, [f"{n}/bias" for n in names]), bank_pre, d.max_k, C)
    else:
        for k in range(1, d.max_k + 1):
            sc = names[k - 1]
            K.conv1d(inp, P[f"{sc}/kernel"], P[f"{sc}/bias"], out=bank_pre[:, :, (k - 1) * C:k * C])
    bank = torch.empty_like(bank_pre)
    gam = _contig_span(P, [f"{n}/bn/gamma" for n in names])
    bet = _contig_span(P, [f"{n}/bn/beta" for n in names])
    mp = torch.empty_like(bank)
    # BN + ReLU and the max-pool (module.py:79-80) in one pass over the bank
    fused = os.environ.get("SAT_BANK_POOL_FUSED", "1") == "1"       # 0: two launches (A/B)
    st_bank = _bn(bank_pre.view(-1, KC), bank.view(-1, KC), gam, bet, bn, f"{names[0]}/bn", KC, True,
                  training, ws, pool=(bank_pre, bank, mp) if fused else None)
    if not fused:
        K.maxpool2(bank, mp)                                          # module.py:80
    p1_pre = K.conv1d(mp, P["encoder/cbhg/proj1/kernel"], P["encoder/cbhg/proj1/bias"])
    p1 = torch.empty_like(p1_pre)
    st_p1 = _bn(p1_pre.view(-1, d.proj1), p1.view(-1, d.proj1), P["encoder/cbhg/proj1/bn/gamma"],
                P["encoder/cbhg/proj1/bn/beta"], bn, "encoder/cbhg/proj1/bn", d.proj1, True,
                training, ws)
    p2_pre = K.conv1d(p1, P["encoder/cbhg/proj2/kernel"], P["encoder/cbhg/proj2/bias"])
    hw = torch.empty_like(p2_pre)                                     # BN(proj2) + residual
    st_p2 = _bn(p2_pre.view(-1, d.proj2), hw.view(-1, d.proj2), P["encoder/cbhg/proj2/bn/gamma"],
                P["encoder/cbhg/proj2/bn/beta"], bn, "encoder/cbhg/proj2/bn", d.proj2, False,
                training, ws, res=inp.view(-1, d.proj2))
    sv.update(bank_pre=bank_pre, bank=bank, mp=mp, p1_pre=p1_pre, p1=p1, p2_pre=p2_pre,
              st_bank=st_bank, st_p1=st_p1, st_p2=st_p2)
    if d.needs_adjust:                                                # module.py:88-89
        sv["hw_in_adjust"] = hw
        hw = K.linear(hw, P["encoder/cbhg/adjustment/kernel"], P["encoder/cbhg/adjustment/bias"])
    hws = [hw]
    for i in range(d.num_highway):                                    # ext HighwayNet
        sc = f"encoder/cbhg/highway{i}"
        y = torch.empty_like(hw)
        Wp = K.pair_view(P[f"{sc}/H/kernel"], P[f"{sc}/T/kernel"])
        bp = K.pair_view(P[f"{sc}/H/bias"], P[f"{sc}/T/bias"])
        if Wp is not None and bp is not None and Wp[1] == bp[1]:
            # H and T pre-activations as ONE batched product (the two weights / biases are a
            # constant distance apart in the parameter arena), activations fused into the combine
            ht = torch.empty(2, *hw.shape, device=dev)
            K.gemm(hw.reshape(-1, hw.shape[-1]), Wp[0], ht.view(2, -1, hw.shape[-1]),
                   bias=bp[0].view(2, -1))
            h, t = (ht[1], ht[0]) if Wp[1] else (ht[0], ht[1])
            K.highway_act_fwd(h, t, hw, y)
        else:
            h = K.linear(hw, P[f"{sc}/H/kernel"], P[f"{sc}/H/bias"], act="relu")
            t = K.linear(hw, P[f"{sc}/T/kernel"], P[f"{sc}/T/bias"], act="sigmoid")
            K.highway_fwd(h, t, hw, y)
        hws.append((h, t, y))
        hw = y
    sv["hws"] = hws
    # bidirectional ZoneoutLSTM (module.py:93-110): outputs written straight into M1 halves
    U = d.cbhg_half
    m1 = torch.empty(B, N, 2 * U, device=dev)
    zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
    # the two directions are independent recurrences: step n of the forward cell and step
    # N-1-n of the backward cell run as ONE multi-problem launch (sat_lstm_steps_fwd)
    lstm = {}
    zs = K.zeros_group(*([(N + 1, B, U)] * 4), device=dev)   # c / h histories, one fill
    Win = hw.shape[-1]
    Wp = K.pair_view(P["encoder/cbhg/lstm_fw/kernel"][:Win], P["encoder/cbhg/lstm_bw/kernel"][:Win])
    bp = K.pair_view(P["encoder/cbhg/lstm_fw/bias"], P["encoder/cbhg/lstm_bw/bias"])
    X = None
    if Wp is not None and bp is not None and Wp[1] == bp[1]:
        # both directions' input projections as ONE batched product
        Xp = torch.empty(2, B, N, 4 * U, device=dev)
        K.gemm(hw.reshape(-1, Win), Wp[0], Xp.view(2, B * N, 4 * U), bias=bp[0].view(2, -1))
        X = (Xp[1], Xp[0]) if Wp[1] else (Xp[0], Xp[1])
    for i, dr in enumerate(("fw", "bw")):
        Wk = P[f"encoder/cbhg/lstm_{dr}/kernel"]
        lstm[dr] = dict(
            X=X[i] if X is not None else K.linear(hw, Wk[:Win], P[f"encoder/cbhg/lstm_{dr}/bias"]),
            CS=zs[2 * i], HS=zs[2 * i + 1],                       # X: [B, N, 4U]
            G=torch.empty(N, B, 4 * U, device=dev))

    def enc_step(dr, rev, n):
        st = lstm[dr]
        Wk = P[f"encoder/cbhg/lstm_{dr}/kernel"]
        mc, mh = mk(f"enc/lstm_{dr}/zc"), mk(f"enc/lstm_{dr}/zh")
        out = m1[:, :, U:] if rev else m1[:, :, :U]
        prev, nxt = (n + 1, n) if rev else (n, n + 1)
        return dict(B=B, U=U, K=U, t=n, xproj=st["X"][:, n], rin=st["HS"][prev],
                    W=Wk[hw.shape[-1]:], c_prev=st["CS"][prev], h_prev=st["HS"][prev],
                    mask_c=None if mc is None else mc[n], mask_h=None if mh is None else mh[n],
                    zc=zc, zh=zh, h_raw=out[:, n], c_out=st["CS"][nxt], h_out=st["HS"][nxt],
                    gates=st["G"][n], lengths=lengths)

    sv["enc_persistent"] = persistent and U == 128
    if before_lstm is not None:
        before_lstm()
    if sv["enc_persistent"]:
        # all N steps of both directions in ONE launch (encoder_lstm.hip: one workgroup per
        # (direction, utterance) keeps the recurrent matrix in registers)
        mcs = {dr: (mk(f"enc/lstm_{dr}/zc"), mk(f"enc/lstm_{dr}/zh")) for dr in ("fw", "bw")}
        X = lstm["fw"]["X"]
        K.encoder_lstm_fwd(
            B=B, N=N, U=U, zc=zc, zh=zh, X_fw=lstm["fw"]["X"], X_bw=lstm["bw"]["X"],
            x_sb=X.stride(0), x_sn=X.stride(1),
            W_fw=P["encoder/cbhg/lstm_fw/kernel"][hw.shape[-1]:],
            W_bw=P["encoder/cbhg/lstm_bw/kernel"][hw.shape[-1]:],
            mc_fw=mcs["fw"][0], mh_fw=mcs["fw"][1], mc_bw=mcs["bw"][0], mh_bw=mcs["bw"][1],
            lengths=lengths, H=m1, h_sb=m1.stride(0), h_sn=m1.stride(1),
            CS_fw=lstm["fw"]["CS"], HS_fw=lstm["fw"]["HS"], CS_bw=lstm["bw"]["CS"],
            HS_bw=lstm["bw"]["HS"], G_fw=lstm["fw"]["G"], G_bw=lstm["bw"]["G"])
    else:
        for n in range(N):
            K.lstm_steps_fwd([enc_step("fw", False, n), enc_step("bw", True, N - 1 - n)])
    sv["enc_lstm"] = lstm
    sv["m1"] = m1
    s0 = K.linear(m1, P["encoder/self_attention_projection/kernel"],
                  P["encoder/self_attention_projection/bias"])          # module.py:429
    x = s0
    sv["s0"] = s0
    for h in range(d.enc_hops):
        x = sa_transformer_fwd(x, P, f"encoder/self_attention{h}", d.enc_heads, False,
                               mk(f"enc/sa{h}/probs"), sv, f"enc_sa{h}")
    return m1, x


def _bn(x2, y2, gamma, beta, bn: BNState, scope, C, relu, training, ws, res=None, pool=None):
    """``pool`` = (x3, y3, mp3): also the max-pool of the output into mp3, fused (no ``res``)."""
    dev = x2.device
    if training:
        mean = torch.empty(C, device=dev)
        var = torch.empty(C, device=dev)
        mm, mv = bn.span(scope, C)
        K.bn_stats(x2, mean, var, ws, mm, mv, momentum=0.99)
    else:
        mean, var = bn.span(scope, C)
    if pool is not None:
        K.bn_apply_maxpool2(*pool, mean, var, gamma, beta, relu=relu)
    else:
        K.bn_apply(x2, y2, mean, var, gamma, beta, relu=relu, res=res)
    return dict(mean=mean, var=var, gamma=gamma, beta=beta)


def head_fwd(P, hp, d: PR.Dims, dout_sm: torch.Tensor, masks, sv):
    """RNNTransformer training-branch tail (modules/module.py:754-764)."""
    Tp, B, Dd = dout_sm.shape
    mk = (lambda n: masks[n]) if masks is not None else (lambda n: None)
    D = K.contiguous(dout_sm.transpose(0, 1))                         # [B, T', D] (data movement)
    z = D
    for h in range(d.dec_hops):
        z = sa_transformer_fwd(z, P, f"decoder/self_attention{h}", d.dec_heads, True,
                               mk(f"dec/sa{h}/probs"), sv, f"dec_sa{h}")
    mel = K.linear(z, P["decoder/out_projection/kernel"], P["decoder/out_projection/bias"])
    stop = K.linear(z, P["decoder/stop_token_projection/kernel"],
                    P["decoder/stop_token_projection/bias"])
    sv.update(D=D, Z=z)
    return mel, stop


class Saved(dict):
    pass


def model_forward(P, bn: BNState, hp, d: PR.Dims, batch: Dict[str, torch.Tensor],
                  masks: Optional[Dict[str, torch.Tensor]], training: bool, ws: K.Workspace,
                  compute_grad_seeds: bool = True, attn_tile: int = 32, pipe=None,
                  persistent: bool = False, scratch=None,
                  health: Optional[torch.Tensor] = None):
    """model_fn forward + loss.  Returns (outputs dict, Saved).  ``health``: the engine's int32
    error arena -- words 8 and 9 take the embedding / speaker-embedding id-range flags."""
    sv = Saved()
    ids, lengths = batch["source"], batch["source_length"]
    # the decoder's target-only inputs (prenets, the attention RNN's input projection) on a
    # second stream beside the encoder, whose BiLSTM holds only 64 CUs (persistent path, single
    # speaker); joined before the decoder reads them
    aux, fork = None, None
    dec_box = [None]
    if persistent and not d.multi_speaker and ids.is_cuda:
        aux = K.aux_stream(ids.device)

        def fork():      # forked at the BiLSTM launch: it fills the CUs the BiLSTM leaves idle
            dec_box[0] = decoder_inputs(P, hp, d, batch["mel"], masks, aux,
                                        N=batch["source"].shape[1])
    m1, m2 = encoder_fwd(P, bn, hp, d, ids, lengths, masks, training, ws, sv,
                         persistent=persistent, err=None if health is None else health[8:9],
                         before_lstm=fork)
    dec_in = dec_box[0]
    if aux is not None:
        torch.cuda.current_stream().wait_stream(aux)
    spk = None
    if d.multi_speaker:                                               # models/models.py:43-46,69
        ids_s = batch["speaker_id"]
        spk = torch.empty(ids_s.shape[0], d.spk_dim, device=m1.device)
        if health is None:
            sv["spk_err"] = K.zeros(1, dtype=torch.int32, device=m1.device)
        else:
            sv["spk_err"] = K.fill_(health[9:10])
        K.embedding_fwd(P["speaker_embedding"], ids_s, spk, d.spk_offset, sv["spk_err"])
    dout, dsv = decoder_forward(P, hp, d, m1, m2, lengths, batch["mel"], masks,
                                attn_tile=attn_tile, spk=spk, persistent=persistent,
                                scratch=scratch, keep_tanh=compute_grad_seeds, inputs=dec_in,
                                **({} if pipe is None else {"pipe": pipe}))
    sv["dec"] = dsv
    if spk is not None:
        dsv.tensors["ms_prenet"]["ids"] = batch["speaker_id"]
    mel_r, stop = head_fwd(P, hp, d, dout, masks, sv)
    B, Tp, _ = mel_r.shape
    mel = mel_r.view(B, Tp * d.r, d.num_mels)                         # module.py:1561
    loss = torch.empty(8, device=m1.device)          # sat_loss_fwd_bwd writes [0:5]; [5:8] unused
    dmel = dstop = None
    if compute_grad_seeds:
        dmel = torch.empty_like(mel)
        dstop = torch.empty(B, Tp, device=m1.device)
    K.loss_fwd_bwd(mel, batch["mel"], batch["mel_mask"], stop.view(B, Tp), batch["done"],
                   batch["done_mask"], loss, dmel, dstop)
    sv.update(mel=mel, stop=stop, dmel=dmel, dstop=dstop, m2=m2, batch=batch, masks=masks,
              training=training)
    out = {"mel": mel, "stop": stop, "loss": loss[0:1], "l1": loss[1:2], "bce": loss[2:3],
           "m1": m1, "m2": m2, "dout": dout, "alignment1": dsv.AL1[1:], "alignment2": dsv.S2}
    return out, sv
