"""CPU ORACLE -- test infrastructure only.

A plain restatement of the reference's teacher-forced Self-attention Tacotron step
(rhoposit/self-attention-tacotron, TF1.x) in float64 PyTorch-CPU ops, step-wise like
``tf.contrib.seq2seq.dynamic_decode``.  PyTorch is used here only as a CPU array library with
autograd (the gradients of this restatement are the parity reference for the HIP backward).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product path never calls it.

PARITY STATUS: the reference cannot run in this container (no TensorFlow 1.x, no tacotron2
dependency, no network -- SURVEY.md section 8(c)).  The reference ships no golden vectors; the
only behavioural test it holds is ``modules/transformer_test.py:44-90`` (training branch ==
teacher-forced incremental branch), which ``tests/test_oracle.py`` reproduces.  Everything that
lives in TF / tacotron2@6af04c7 (LSTMCell, zoneout, Conv1d+BN, HighwayNet, PreNet, losses) is
restated from their published semantics => **parity unpinned** against
true TF numbers for those rows.

Masks: training-mode randomness (dropout, zoneout) is an INPUT (``masks`` dict, names from
``masks.mask_specs``), so the GPU path and this oracle can be fed identical masks.
``masks=None`` selects the deterministic eval semantics (no dropout, zoneout blend, BN moving
statistics) -- the reference's ``loss_with_teacher`` computation.
"""

from __future__ import annotations

import math
from typing import Dict, Optional

import torch

Tensor = torch.Tensor


# ----------------------------------------------------------------------------- generic layers

def dense(x: Tensor, p: Dict[str, Tensor], scope: str, act=None) -> Tensor:
    """tf.layers.Dense: y = x @ W + b (W [in, out])."""
    y = x @ p[f"{scope}/kernel"]
    b = p.get(f"{scope}/bias")
    if b is not None:
        y = y + b
    return act(y) if act is not None else y


def conv1d_same(x: Tensor, w: Tensor, b: Optional[Tensor]) -> Tensor:
    """tf.layers.Conv1D(padding='SAME', stride 1): pad_left=(k-1)//2, pad_right=k-1-pad_left,
    cross-correlation, kernel [k, Cin, Cout].  x [B, N, Cin] -> [B, N, Cout]."""
    k = w.shape[0]
    pl = (k - 1) // 2
    pr = k - 1 - pl
    B, N, C = x.shape
    xp = torch.cat([x.new_zeros(B, pl, C), x, x.new_zeros(B, pr, C)], dim=1)
    y = 0
    for j in range(k):
        y = y + xp[:, j:j + N, :] @ w[j]
    return y + b if b is not None else y


def batch_norm(x: Tensor, p: Dict[str, Tensor], bufs: Optional[Dict[str, Tensor]], scope: str,
               training: bool, eps: float = 1e-3) -> Tensor:
    """tf.layers.BatchNormalization (axis -1, eps 1e-3).  Training: biased batch moments over
    every (b, n) position including padding.  Eval: moving statistics."""
    g, be = p[f"{scope}/gamma"], p[f"{scope}/beta"]
    if training:
        mean = x.mean(dim=(0, 1))
        var = ((x - mean) ** 2).mean(dim=(0, 1))
    else:
        mean = bufs[f"{scope}/moving_mean"]
        var = bufs[f"{scope}/moving_variance"]
    return g * (x - mean) / torch.sqrt(var + eps) + be


def conv_bn(x, p, bufs, scope, training, relu: bool):
    """ext tacotron2 Conv1d: Conv1D(SAME, bias) -> BatchNormalization -> activation
    (drop_rate 0 in CBHG).  Called at modules/module.py:46-68."""
    y = conv1d_same(x, p[f"{scope}/kernel"], p[f"{scope}/bias"])
    y = batch_norm(y, p, bufs, f"{scope}/bn", training)
    return torch.relu(y) if relu else y


def maxpool2_same(x: Tensor) -> Tensor:
    """MaxPooling1D(pool 2, stride 1, SAME) (modules/module.py:54): out[n]=max(x[n],x[n+1]),
    out[N-1]=x[N-1]."""
    nxt = torch.cat([x[:, 1:, :], x[:, -1:, :]], dim=1)
    return torch.maximum(x, nxt)


def prenet(x, p, scope, mask: Optional[Tensor]):
    """ext tacotron2 PreNet: dropout_{0.5}(ReLU(Dense(x))); mask holds 0 or 1/keep."""
    y = dense(x, p, scope, torch.relu)
    return y * mask if mask is not None else y


def lstm_cell(x, c, h, w, b, forget_bias: float = 1.0):
    """TF LSTMCell: [i, j, f, o] = [x; h] @ W + b; c' = s(f+1)c + s(i)tanh(j); h' = s(o)tanh(c')."""
    z = torch.cat([x, h], dim=-1) @ w + b
    i, j, f, o = torch.chunk(z, 4, dim=-1)
    c_new = torch.sigmoid(f + forget_bias) * c + torch.sigmoid(i) * torch.tanh(j)
    h_new = torch.sigmoid(o) * torch.tanh(c_new)
    return h_new, c_new


def zoneout_lstm_step(x, c, h, w, b, zc: float, zh: float, mc: Optional[Tensor],
                      mh: Optional[Tensor]):
    """ext tacotron2 ZoneoutLSTMCell.  Training with keep-masks m:
    c = m_c*c' + (1-m_c)*c, h = m_h*h' + (1-m_h)*h  (== (1-z)*dropout_{1-z}(x'-x) + x).
    Eval: c = (1-z_c)c' + z_c c, h = (1-z_h)h' + z_h h.  The cell OUTPUT is the raw h'."""
    h_raw, c_raw = lstm_cell(x, c, h, w, b)
    if mc is not None:
        c2 = mc * c_raw + (1.0 - mc) * c
        h2 = mh * h_raw + (1.0 - mh) * h
    else:
        c2 = (1.0 - zc) * c_raw + zc * c
        h2 = (1.0 - zh) * h_raw + zh * h
    return h_raw, c2, h2


def mha(x: Tensor, p, scope: str, heads: int, causal: bool, probs_mask: Optional[Tensor]):
    """modules/self_attention.py:108-128 + ScaledDotProductAttentionMechanism :45-65.
    Q,K,V = Dense(model)(x) split into heads; softmax(QK^T/sqrt(head_dim)); NO padding mask
    (use_padding_mask False, module.py:353-356); causal mask -> -inf above the diagonal;
    dropout on probs (training); output_projection.  Returns (out, probs)."""
    B, L, _ = x.shape
    q = dense(x, p, f"{scope}/query_projection")
    k = dense(x, p, f"{scope}/key_projection")
    v = dense(x, p, f"{scope}/value_projection")
    model = q.shape[-1]
    dh = model // heads

    def split(t):
        return t.view(B, L, heads, dh).transpose(1, 2)

    q, k, v = split(q), split(k), split(v)
    s = q @ k.transpose(-1, -2) / math.sqrt(dh)
    if causal:
        m = torch.ones(L, L, dtype=torch.bool).triu(1)
        s = s.masked_fill(m, float("-inf"))
    a = torch.softmax(s, dim=-1)
    ad = a * probs_mask if probs_mask is not None else a
    o = (ad @ v).transpose(1, 2).reshape(B, L, model)
    return dense(o, p, f"{scope}/output_projection"), a


def sa_transformer(x, p, scope, heads, causal, probs_mask):
    """SelfAttentionTransformer.call (modules/module.py:363-371): x + tanh(Dense(MHA(x)))."""
    y, a = mha(x, p, f"{scope}/mha", heads, causal, probs_mask)
    return x + dense(y, p, f"{scope}/transform", torch.tanh), a


# ----------------------------------------------------------------------------- encoder

def lstm_sequence(x, lengths, w, b, zc, zh, mc, mh, reverse: bool):
    """One direction of bidirectional_dynamic_rnn(sequence_length) with a ZoneoutLSTMCell.
    Forward: outputs 0 and state frozen for t >= len.  Backward: runs over the reversed valid
    prefix (reverse_sequence), outputs re-reversed, 0 past len.  Masks are indexed by the time
    position n ([N, B, U])."""
    B, N, _ = x.shape
    U = b.shape[0] // 4
    c = x.new_zeros(B, U)
    h = x.new_zeros(B, U)
    outs = [None] * N
    order = range(N - 1, -1, -1) if reverse else range(N)
    for n in order:
        valid = (n < lengths).to(x.dtype).unsqueeze(1)
        out, c2, h2 = zoneout_lstm_step(x[:, n], c, h, w, b, zc, zh,
                                        None if mc is None else mc[n],
                                        None if mh is None else mh[n])
        c = valid * c2 + (1 - valid) * c
        h = valid * h2 + (1 - valid) * h
        outs[n] = out * valid
    return torch.stack(outs, dim=1)


def encoder(ids, lengths, p, bufs, hp, masks, training, kinks=None):
    """SelfAttentionCBHGEncoder.call (modules/module.py:425-438) -> (M1, M2, alignments).

    ``kinks`` (tests only): the branch another implementation took at every piecewise-linear
    point of the encoder front -- {"prenet{i}": relu gate, "bank": conv-bank relu gate,
    "pool_first": max-pool window choice (out[n] takes x[n]), "proj1": relu gate} as 0/1
    tensors.  The float64 arithmetic then follows the same sub-gradient branch, so a gradient
    comparison measures rounding, not which side of a kink fp32 and fp64 landed on (a gate that
    flips routes an element's whole gradient differently).  The forward values change only by
    the flipped elements' distance from the kink (fp32 rounding)."""
    g = (lambda k: masks[k]) if masks is not None else (lambda k: None)
    kk = kinks or {}
    x = p["embedding"][ids]                                           # ext Embedding
    for i in range(len(hp.encoder_prenet_out_units)):
        if f"prenet{i}" in kk:
            x = dense(x, p, f"encoder/prenet{i}") * kk[f"prenet{i}"]
            m = g(f"enc/prenet{i}")
            x = x * m if m is not None else x
        else:
            x = prenet(x, p, f"encoder/prenet{i}", g(f"enc/prenet{i}"))
    inp = x
    if "bank" in kk:
        z = torch.cat([conv_bn(x, p, bufs, f"encoder/cbhg/conv_bank/K{k}", training, relu=False)
                       for k in range(1, hp.max_filter_width + 1)], dim=-1) * kk["bank"]
        nxt = torch.cat([z[:, 1:, :], z[:, -1:, :]], dim=1)
        y = torch.where(kk["pool_first"].bool(), z, nxt)
    else:
        bank = [conv_bn(x, p, bufs, f"encoder/cbhg/conv_bank/K{k}", training, relu=True)
                for k in range(1, hp.max_filter_width + 1)]           # module.py:78
        y = maxpool2_same(torch.cat(bank, dim=-1))                    # :80
    if "proj1" in kk:
        y = conv_bn(y, p, bufs, "encoder/cbhg/proj1", training, relu=False) * kk["proj1"]
    else:
        y = conv_bn(y, p, bufs, "encoder/cbhg/proj1", training, relu=True)   # :82
    y = conv_bn(y, p, bufs, "encoder/cbhg/proj2", training, relu=False)  # :83
    y = y + inp                                                       # :86
    if "encoder/cbhg/adjustment/kernel" in p:                         # :88-89
        y = dense(y, p, "encoder/cbhg/adjustment")
    for i in range(hp.num_highway):                                   # :91, ext HighwayNet
        hh = dense(y, p, f"encoder/cbhg/highway{i}/H", torch.relu)
        tt = dense(y, p, f"encoder/cbhg/highway{i}/T", torch.sigmoid)
        y = hh * tt + y * (1.0 - tt)
    zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
    fw = lstm_sequence(y, lengths, p["encoder/cbhg/lstm_fw/kernel"], p["encoder/cbhg/lstm_fw/bias"],
                       zc, zh, g("enc/lstm_fw/zc"), g("enc/lstm_fw/zh"), reverse=False)
    bw = lstm_sequence(y, lengths, p["encoder/cbhg/lstm_bw/kernel"], p["encoder/cbhg/lstm_bw/bias"],
                       zc, zh, g("enc/lstm_bw/zc"), g("enc/lstm_bw/zh"), reverse=True)
    m1 = torch.cat([fw, bw], dim=-1)                                  # :110
    s = dense(m1, p, "encoder/self_attention_projection")             # :429
    aligns = []
    for h in range(hp.self_attention_num_hop):
        s, a = sa_transformer(s, p, f"encoder/self_attention{h}", hp.self_attention_num_heads,
                              False, g(f"enc/sa{h}/probs"))
        aligns.append(a)
    return m1, s, aligns


def encoder_front_branches(ids, p, bufs, hp, masks, training):
    """The oracle's OWN branch at every kink ``encoder(kinks=)`` can be handed (tests only):
    the same keys and the same definitions as the test's record of the HIP forward (prenet
    outputs after dropout > 0, conv-bank ReLU outputs > 0, max-pool ``out[n] = x[n]`` choice on
    the ReLU outputs, proj1 ReLU output > 0), so the two can be compared element by element and
    the number of branches that fp32 and float64 take differently is bounded
    (modules/module.py:77-83 front, ext PreNet)."""
    g = (lambda k: masks[k]) if masks is not None else (lambda k: None)
    x = p["embedding"][ids]
    out = {}
    for i in range(len(hp.encoder_prenet_out_units)):
        x = prenet(x, p, f"encoder/prenet{i}", g(f"enc/prenet{i}"))
        out[f"prenet{i}"] = x > 0
    bank = torch.cat([conv_bn(x, p, bufs, f"encoder/cbhg/conv_bank/K{k}", training, relu=True)
                      for k in range(1, hp.max_filter_width + 1)], dim=-1)
    nxt = torch.cat([bank[:, 1:, :], bank[:, -1:, :]], dim=1)
    out["bank"] = bank > 0
    out["pool_first"] = bank >= nxt
    y = conv_bn(torch.maximum(bank, nxt), p, bufs, "encoder/cbhg/proj1", training, relu=True)
    out["proj1"] = y > 0
    return {k: v.double() for k, v in out.items()}


# ----------------------------------------------------------------------------- attention

def seq_mask(lengths, n, dtype):
    return (torch.arange(n).unsqueeze(0) < lengths.unsqueeze(1)).to(dtype)


class ForwardAttentionOracle:
    """modules/forward_attention.py:48-136 on top of TF BahdanauAttention's memory handling."""

    def __init__(self, p, scope, memory, lengths):
        self.p, self.scope = p, scope
        mask = seq_mask(lengths, memory.shape[1], memory.dtype)
        self.values = memory * mask.unsqueeze(-1)                     # _prepare_memory
        self.keys = self.values @ p[f"{scope}/memory_layer/kernel"]
        self.mask = mask.bool()

    def initial_state(self, B, N, dtype):                             # :128-136
        s0 = torch.zeros(B, N, dtype=dtype)
        a0 = torch.cat([torch.ones(B, 1, dtype=dtype), torch.zeros(B, N - 1, dtype=dtype)], 1)
        u0 = 0.5 * torch.ones(B, 1, dtype=dtype)
        return s0, a0, u0

    def __call__(self, query, state):                                 # :88-122
        prev_s, prev_a, u = state
        p, sc = self.p, self.scope
        q = query @ p[f"{sc}/query_layer/kernel"]                     # :92
        f = conv1d_same(prev_s.unsqueeze(-1), p[f"{sc}/location_conv/kernel"],
                        p[f"{sc}/location_conv/bias"])                # :98-100
        loc = f @ p[f"{sc}/location_layer/kernel"]                    # :101
        e = (p[f"{sc}/attention_variable"] *
             torch.tanh(self.keys + q.unsqueeze(1) + loc + p[f"{sc}/attention_bias"])).sum(-1)
        e = e.masked_fill(~self.mask, float("-inf"))                  # _maybe_mask_score
        s = torch.softmax(e, dim=-1)                                  # :105
        shifted = torch.cat([torch.zeros_like(prev_a[:, :1]), prev_a[:, :-1]], dim=1)
        a = ((1 - u) * prev_a + u * shifted + 1e-7) * s               # :108-109
        a = a / a.sum(dim=1, keepdim=True)                            # :110
        return a, (s, a, u)                                           # :116-121


class AdditiveAttentionOracle:
    """TF BahdanauAttention(num_units, normalize=False), built at modules/attentions.py:53-57."""

    def __init__(self, p, scope, memory, lengths):
        self.p, self.scope = p, scope
        mask = seq_mask(lengths, memory.shape[1], memory.dtype)
        self.values = memory * mask.unsqueeze(-1)
        self.keys = self.values @ p[f"{scope}/memory_layer/kernel"]
        self.mask = mask.bool()

    def initial_state(self, B, N, dtype):
        return torch.zeros(B, N, dtype=dtype)

    def __call__(self, query, state):
        p, sc = self.p, self.scope
        q = query @ p[f"{sc}/query_layer/kernel"]
        e = (p[f"{sc}/attention_v"] * torch.tanh(self.keys + q.unsqueeze(1))).sum(-1)
        e = e.masked_fill(~self.mask, float("-inf"))
        s = torch.softmax(e, dim=-1)
        return s, s


def make_attention(kind, p, scope, memory, lengths):
    """attention_mechanism_factory dispatch (modules/attentions.py:25-62)."""
    if kind == "forward":
        return ForwardAttentionOracle(p, scope, memory, lengths)
    if kind == "additive":
        return AdditiveAttentionOracle(p, scope, memory, lengths)
    raise ValueError(f"Unknown attention mechanism: {kind}")


# ----------------------------------------------------------------------------- decoder

def teacher_inputs(targets, r, n_feed):
    """TransformerTrainingHelper (modules/helpers.py:13-58): step 0 = zeros (go frame),
    step t>0 = targets.reshape(B, T/r, mels*r)[:, t-1, -mels*n_feed:]."""
    B, T, M = targets.shape
    g = targets.reshape(B, T // r, M * r)
    go = targets.new_zeros(B, 1, M * n_feed)
    return torch.cat([go, g[:, :-1, -M * n_feed:]], dim=1)            # [B, T', M*n_feed]


def decoder_prenets(x, p, hp, masks, spk):
    # decoder prenet masks are stored step-major [T', B, u]; x is [B, T', .]
    g = (lambda k: masks[k].transpose(0, 1)) if masks is not None else (lambda k: None)
    n = len(hp.decoder_prenet_out_units)
    if spk is not None:                                               # multi_speaker_modules.py:27-32
        d0 = dense(x, p, "decoder/prenet0/dense0", torch.relu)
        sp = dense(spk, p, "decoder/prenet0/speaker_projection", torch.nn.functional.softsign)
        d0 = d0 + sp.unsqueeze(1) if d0.dim() == 3 else d0 + sp
        y = dense(d0, p, "decoder/prenet0/dense", torch.relu)
        m = g("dec/prenet0")
        y = y * m if m is not None else y
        start = 1
    else:
        y, start = x, 0
    for i in range(start, n):
        y = prenet(y, p, f"decoder/prenet{i}", g(f"dec/prenet{i}"))
    return y


def decoder_loop(m1, m2, lengths, targets, p, hp, masks, spk=None, record=False):
    """DualSourceTransformerDecoder.call -> RNNTransformer (training branch) loop part:
    dynamic_decode over T' = T/r steps of DecoderRNNV2 = MultiRNNCell([DualSourceAttentionRNN,
    ZLSTM, ZLSTM]) (modules/module.py:1499-1547, 743-747).  Returns D [B, T', dec] (the raw h2'
    outputs) and the alignment histories."""
    g = (lambda k: masks[k]) if masks is not None else (lambda k: None)
    B, N, _ = m1.shape
    r, nf = hp.outputs_per_step, hp.n_feed_frame
    x = teacher_inputs(targets, r, nf)
    Tp = x.shape[1]
    pre = decoder_prenets(x, p, hp, masks, spk)                       # prenets are per-frame
    att1 = make_attention(hp.attention, p, "decoder/attention1", m1, lengths)
    att2 = make_attention(hp.attention2, p, "decoder/attention2", m2, lengths)
    dt = m1.dtype
    A, D = hp.attention_out_units, hp.decoder_out_units
    st1 = att1.initial_state(B, N, dt)
    st2 = att2.initial_state(B, N, dt)
    c1 = m1.new_zeros(B, m1.shape[2])
    c2 = m2.new_zeros(B, m2.shape[2])
    c0 = h0 = m1.new_zeros(B, A)
    cc1 = hh1 = m1.new_zeros(B, D)
    cc2 = hh2 = m1.new_zeros(B, D)
    zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
    outs, al1, al2 = [], [], []
    rec = {"h0": [], "c1": [], "c2": [], "h1": [], "q": []} if record else None
    for t in range(Tp):
        def mk(name):
            m = g(name)
            return None if m is None else m[t]
        # AttentionWrapper: cell input = concat(inputs, previous attention)
        cell_in = torch.cat([pre[:, t], c1, c2], dim=-1)
        h0_out, c0, h0 = zoneout_lstm_step(cell_in, c0, h0, p["decoder/attention_lstm/kernel"],
                                           p["decoder/attention_lstm/bias"], zc, zh,
                                           mk("dec/lstm0/zc"), mk("dec/lstm0/zh"))
        a1, st1 = att1(h0_out, st1)
        a2, st2 = att2(h0_out, st2)
        c1 = (a1.unsqueeze(1) @ att1.values).squeeze(1)               # _compute_attention
        c2 = (a2.unsqueeze(1) @ att2.values).squeeze(1)
        o = torch.cat([h0_out, c1, c2], dim=-1)                       # ConcatOutputAndAttention
        h1_out, cc1, hh1 = zoneout_lstm_step(o, cc1, hh1, p["decoder/lstm1/kernel"],
                                             p["decoder/lstm1/bias"], zc, zh,
                                             mk("dec/lstm1/zc"), mk("dec/lstm1/zh"))
        h2_out, cc2, hh2 = zoneout_lstm_step(h1_out, cc2, hh2, p["decoder/lstm2/kernel"],
                                             p["decoder/lstm2/bias"], zc, zh,
                                             mk("dec/lstm2/zc"), mk("dec/lstm2/zh"))
        outs.append(h2_out)
        al1.append(a1)
        al2.append(a2)
        if record:
            rec["h0"].append(h0_out)
            rec["c1"].append(c1)
            rec["c2"].append(c2)
            rec["h1"].append(h1_out)
    out = torch.stack(outs, dim=1)
    extra = {"alignment1": torch.stack(al1, 1), "alignment2": torch.stack(al2, 1)}
    if record:
        for k, v in rec.items():
            if v:
                extra[k] = torch.stack(v, 1)
    return out, extra


def decoder_head(dout, p, hp, masks):
    """RNNTransformer training branch tail (modules/module.py:754-764): causal self-attention
    hops, then out_projection [dsa -> mels*r] and stop_token_projection [dsa -> 1]."""
    g = (lambda k: masks[k]) if masks is not None else (lambda k: None)
    z = dout
    for h in range(hp.decoder_self_attention_num_hop):
        z, _ = sa_transformer(z, p, f"decoder/self_attention{h}",
                              hp.decoder_self_attention_num_heads, True, g(f"dec/sa{h}/probs"))
    mel = dense(z, p, "decoder/out_projection")
    stop = dense(z, p, "decoder/stop_token_projection")
    return mel, stop, z


def decoder_head_incremental(dout, p, hp):
    """Eval-time TransformerWrapper path (modules/rnn_wrappers.py:111-124, :209-214): each step
    re-runs the self-attention over the history and keeps the last row."""
    B, Tp, _ = dout.shape
    mels, stops = [], []
    for t in range(Tp):
        hist = dout[:, :t + 1]
        z = hist
        for h in range(hp.decoder_self_attention_num_hop):
            z, _ = sa_transformer(z, p, f"decoder/self_attention{h}",
                                  hp.decoder_self_attention_num_heads, True, None)
        last = z[:, -1]
        mels.append(dense(last, p, "decoder/out_projection"))
        stops.append(dense(last, p, "decoder/stop_token_projection"))
    return torch.stack(mels, 1), torch.stack(stops, 1)


# ----------------------------------------------------------------------------- loss / model

def losses(mel, stop, targets, target_mask, done, done_mask):
    """models/models.py:159-173: 0.1 * L1(codes_loss, 'l1') + sigmoid xent (binary_loss);
    tf.losses reduction SUM_BY_NONZERO_WEIGHTS."""
    B, T, M = targets.shape
    w = target_mask.unsqueeze(-1).expand(B, T, M)
    l1 = (w * (mel - targets).abs()).sum() / (w != 0).sum().clamp(min=1)
    x = stop.squeeze(-1)
    xent = torch.clamp(x, min=0) - x * done + torch.log1p(torch.exp(-x.abs()))
    bce = (done_mask * xent).sum() / (done_mask != 0).sum().clamp(min=1)
    return 0.1 * l1 + bce, l1, bce


def model_forward(p: Dict[str, Tensor], bufs, hp, batch: Dict[str, Tensor],
                  masks: Optional[Dict[str, Tensor]], training: bool, record=False, kinks=None):
    """model_fn TRAIN/EVAL-with-teacher forward (models/models.py:23-173).  Returns a dict with
    mel [B,T,mels], stop [B,T',1], loss terms and intermediate tensors.  ``kinks``: see
    ``encoder`` (tests only)."""
    m1, m2, enc_al = encoder(batch["source"], batch["source_length"], p, bufs, hp, masks,
                             training, kinks=kinks)
    spk = None
    if hp.use_speaker_embedding and hp.speaker_embedd_to_prenet:
        spk = p["speaker_embedding"][batch["speaker_id"] - hp.speaker_embedding_offset]
    dout, extra = decoder_loop(m1, m2, batch["source_length"], batch["mel"], p, hp, masks, spk,
                               record=record)
    mel_r, stop, z = decoder_head(dout, p, hp, masks)
    B = mel_r.shape[0]
    mel = mel_r.reshape(B, -1, hp.num_mels)                           # module.py:1561
    loss, l1, bce = losses(mel, stop, batch["mel"], batch["mel_mask"], batch["done"],
                           batch["done_mask"])
    out = {"mel": mel, "stop": stop, "loss": loss, "l1": l1, "bce": bce, "m1": m1, "m2": m2,
           "dout": dout, "z": z}
    out.update(extra)
    return out


def infer_free_running(p: Dict[str, Tensor], bufs, hp, batch: Dict[str, Tensor],
                       max_iters: Optional[int] = None, min_iters: int = 10,
                       forced: Optional[tuple] = None, feed: str = "mel",
                       helper: Optional[str] = None):
    """PREDICT branch of model_fn (models/models.py:84-97, 252-277) with the inference decoder
    of RNNTransformer (modules/module.py:766-784): dynamic_decode over
    OutputAndStopTokenTransparentWrapper(TransformerWrapper(RNNStateHistoryWrapper(DecoderRNNV2)))
    driven by the tacotron2 StopTokenBasedInferenceHelper (analog modules/helpers.py:111-160):
      * step 0 input = go frame (zeros); step t+1 input = mel_t[:, -num_mels*n_feed:] (the last
        predicted frame of the r-group);
      * every step appends h2_t to the state history and re-runs the causal self-attention
        transformer over the whole history, keeping the last row (rnn_wrappers.py:111-124);
        mel_t / stop_t are the out / stop-token projections of that row (:209-214);
      * finished after step t iff t > min_iters and sigmoid(stop_t) > 0.5 for EVERY utterance
        (reduce_all); the loop also ends at max_iters (hparams max_iters, JSON 500).
    Eval semantics throughout: no dropout (apply_dropout_on_inference=False, hparams.py:105),
    zoneout blend, BatchNorm moving statistics.  Returns mel [B, T_out*r, mels], stop
    [B, T_out], alignments, the decoder-self-attention probabilities of the last step and
    T_out (the number of decoder steps run).

    ``forced=(A1, A2)`` ([B, T', N] each) restates the forced-alignment second pass
    (models/models.py:118-148): the mechanisms are TeacherForcing{Forward,Additive}Attention
    (modules/teacher_forcing_attention.py:30-35: step t returns A[:, t], the query is unused),
    the helper OneHotValidationHelper(teacher_forcing=False) (modules/helpers.py:96-108): exactly
    T' steps, no stop-token termination, and with ``feed="softmax"`` step t+1 is fed the softmax
    over the feature bins of each frame of step t's output, last n_feed frames (:100-104).

    ``helper="validation"`` restates OneHotValidationHelper without forced alignments
    (modules/helpers.py:61-108, RNNTransformer with is_validation, modules/module.py:733-738):
    exactly T' = batch["mel"].shape[1] / r steps with the real attention mechanisms, no stop
    termination; ``feed="softmax"`` (teacher_forcing=False, model_fn EVAL's loss) or
    ``feed="target"`` (teacher_forcing=True: step t+1 is fed targets[:, t, -M*n_feed:], :103 --
    the incremental branch modules/transformer_test.py:44-90 compares with training)."""
    max_iters = hp.max_iters if max_iters is None else max_iters
    if forced is not None:
        max_iters = forced[0].shape[1]
        helper = "validation"
    helper = "stop_token" if helper is None else helper
    tg = None
    if helper == "validation" and forced is None:
        max_iters = batch["mel"].shape[1] // hp.outputs_per_step
    if feed == "target":
        assert helper == "validation", "feed='target' is OneHotValidationHelper(teacher_forcing=True)"
        Bt = batch["mel"].shape[0]
        tg = batch["mel"].reshape(Bt, max_iters, -1)
    m1, m2, enc_al = encoder(batch["source"], batch["source_length"], p, bufs, hp, None, False)
    spk = None
    if hp.use_speaker_embedding and hp.speaker_embedd_to_prenet:
        spk = p["speaker_embedding"][batch["speaker_id"] - hp.speaker_embedding_offset]
    lengths = batch["source_length"]
    B, N, _ = m1.shape
    M, r, nf = hp.num_mels, hp.outputs_per_step, hp.n_feed_frame
    att1 = make_attention(hp.attention, p, "decoder/attention1", m1, lengths)
    att2 = make_attention(hp.attention2, p, "decoder/attention2", m2, lengths)
    dt = m1.dtype
    A, D = hp.attention_out_units, hp.decoder_out_units
    st1 = att1.initial_state(B, N, dt)
    st2 = att2.initial_state(B, N, dt)
    c1 = m1.new_zeros(B, m1.shape[2])
    c2 = m2.new_zeros(B, m2.shape[2])
    c0 = h0 = m1.new_zeros(B, A)
    cc1 = hh1 = m1.new_zeros(B, D)
    cc2 = hh2 = m1.new_zeros(B, D)
    zc, zh = hp.zoneout_factor_cell, hp.zoneout_factor_output
    x = m1.new_zeros(B, M * nf)                                        # _go_frames
    hist, mels, stops, al1, al2 = [], [], [], [], []
    probs = None
    for t in range(max_iters):
        pre = decoder_prenets(x, p, hp, None, spk)
        cell_in = torch.cat([pre, c1, c2], dim=-1)
        h0_out, c0, h0 = zoneout_lstm_step(cell_in, c0, h0, p["decoder/attention_lstm/kernel"],
                                           p["decoder/attention_lstm/bias"], zc, zh, None, None)
        if forced is not None:
            a1, a2 = forced[0][:, t], forced[1][:, t]
        else:
            a1, st1 = att1(h0_out, st1)
            a2, st2 = att2(h0_out, st2)
        c1 = (a1.unsqueeze(1) @ att1.values).squeeze(1)
        c2 = (a2.unsqueeze(1) @ att2.values).squeeze(1)
        o = torch.cat([h0_out, c1, c2], dim=-1)
        h1_out, cc1, hh1 = zoneout_lstm_step(o, cc1, hh1, p["decoder/lstm1/kernel"],
                                             p["decoder/lstm1/bias"], zc, zh, None, None)
        h2_out, cc2, hh2 = zoneout_lstm_step(h1_out, cc2, hh2, p["decoder/lstm2/kernel"],
                                             p["decoder/lstm2/bias"], zc, zh, None, None)
        hist.append(h2_out)
        z = torch.stack(hist, dim=1)
        probs = []
        for h in range(hp.decoder_self_attention_num_hop):
            z, a = sa_transformer(z, p, f"decoder/self_attention{h}",
                                  hp.decoder_self_attention_num_heads, True, None)
            probs.append(a)
        last = z[:, -1]
        mel_t = dense(last, p, "decoder/out_projection")              # [B, M*r]
        stop_t = dense(last, p, "decoder/stop_token_projection")[:, 0]
        mels.append(mel_t)
        stops.append(stop_t)
        al1.append(a1)
        al2.append(a2)
        if feed == "softmax":
            x = torch.softmax(mel_t.view(B, r, M), dim=-1).reshape(B, r * M)[:, -M * nf:]
        elif feed == "target":
            x = tg[:, t, -M * nf:]
        else:
            x = mel_t[:, -M * nf:]
        if helper == "stop_token" and t > min_iters and bool((torch.sigmoid(stop_t) > 0.5).all()):
            break
    T_out = len(mels)
    mel = torch.stack(mels, dim=1).reshape(B, T_out * r, M)
    return {"mel": mel, "stop": torch.stack(stops, dim=1), "alignment1": torch.stack(al1, 1),
            "alignment2": torch.stack(al2, 1), "decoder_self_alignments": probs,
            "encoder_self_alignments": enc_al, "steps": T_out, "m1": m1, "m2": m2}


def to_torch(d, dtype=torch.float64):
    out = {}
    for k, v in d.items():
        t = torch.as_tensor(v)
        out[k] = t.to(dtype) if t.is_floating_point() else t
    return out


def learning_rate(init_rate: float, global_step: int, step_factor: int = 1) -> float:
    """models/models.py:284-287 (Noam warm-up, 4000 steps)."""
    warm = 4000.0
    step = float(global_step * step_factor + 1)
    return init_rate * warm ** 0.5 * min(step * warm ** -1.5, step ** -0.5)


def clip_by_global_norm(grads, clip: float = 1.0):
    """tf.clip_by_global_norm: g * clip / max(global_norm, clip)."""
    norm = math.sqrt(sum(float((g.double() ** 2).sum()) for g in grads))
    scale = clip / max(norm, clip)
    return [g * scale for g in grads], norm


def adam_tf(param, grad, m, v, lr, step, b1=0.9, b2=0.999, eps=1e-8):
    """tf.train.AdamOptimizer update (epsilon-hat form): lr_t = lr*sqrt(1-b2^t)/(1-b1^t);
    m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr_t * m / (sqrt(v) + eps)."""
    m = b1 * m + (1 - b1) * grad
    v = b2 * v + (1 - b2) * grad * grad
    lr_t = lr * math.sqrt(1 - b2 ** step) / (1 - b1 ** step)
    return param - lr_t * m / (torch.sqrt(v) + eps), m, v
