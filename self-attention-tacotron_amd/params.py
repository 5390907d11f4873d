"""Parameter inventory of the Self-attention Tacotron hot path and its flat HBM layout.

Every trainable tensor the reference creates on the teacher-forced training path is listed
here under a stable name (TF variable scopes flattened to ``a/b/c``), with the shape the
reference's layer would build (citations next to each group).  Both the CPU oracle and the HIP
path consume the same ``{name: array}`` dict, so parity tests feed identical weights.

On the GPU all parameters live in ONE contiguous fp32 arena (``FlatParams``) and all gradients in
a second arena of the same layout: the global-norm clip, the Adam update and the RCCL gradient
all-reduce are then single launches / single collectives over one buffer.  Each tensor starts on
a 256-byte boundary so vectorised (16 B/lane) loads never straddle tensors.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

ALIGN_FLOATS = 64  # 256 B


@dataclass(frozen=True)
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    init: str = "glorot"      # glorot | zeros | ones | const:<v>
    trainable: bool = True


@dataclass(frozen=True)
class Dims:
    """Resolved layer widths for one hparams set (SURVEY.md section 8 'Resolved hparams')."""
    num_symbols: int
    embed: int
    enc_prenet: Tuple[int, ...]
    conv_ch: int
    max_k: int
    proj1: int
    proj2: int
    cbhg_half: int
    num_highway: int
    needs_adjust: bool
    m1: int               # encoder LSTM output width (memory 1)
    m2: int               # encoder self-attention width (memory 2)
    enc_heads: int
    enc_hops: int
    dec_prenet: Tuple[int, ...]
    feed: int             # num_mels * n_feed_frame
    att_rnn: int          # attention-RNN units
    att1: str
    att2: str
    d1: int
    d2: int
    loc_k: int
    loc_f: int
    dec: int              # decoder LSTM units
    dsa: int              # decoder self-attention width
    dec_heads: int
    dec_hops: int
    num_mels: int
    r: int
    multi_speaker: bool
    num_speakers: int
    spk_dim: int
    spk_offset: int


def resolve_dims(hp) -> Dims:
    if hp.encoder != "SelfAttentionCBHGEncoder":
        raise ValueError(f"Unknown encoder: {hp.encoder}")            # models/models.py:345
    if hp.decoder != "DualSourceTransformerDecoder":
        raise ValueError(f"Unknown decoder: {hp.decoder}")            # models/models.py:367
    if hp.decoder_version != "v2":
        raise NotImplementedError("only decoder_version='v2' (DecoderRNNV2) is on the hot path")
    for a in (hp.attention, hp.attention2):
        if a not in ("forward", "additive"):
            raise NotImplementedError(
                f"attention '{a}' is outside the hot path (SURVEY.md section 2 row 5)")
    if hp.cumulative_weights or hp.use_forward_attention_transition_agent:
        raise NotImplementedError("cumulative_weights / transition agent are not used by the "
                                  "shipped self-attention configs")
    if hp.use_external_speaker_embedding or hp.use_accent_type:
        raise NotImplementedError("external speaker / accent embeddings are out of scope")
    if getattr(hp, "code_loss_type", "l1") != "l1":
        # hparams.py:153 allows 'l1' or 'mse'; the shipped configs use l1 and the loss kernel
        # (sat_loss_fwd_bwd) computes only that -- refuse rather than silently compute L1
        raise NotImplementedError(f"code_loss_type={hp.code_loss_type!r}: only 'l1' is built")
    if getattr(hp, "use_l2_regularization", False):
        # models/models.py:164-171 (ext l2_regularization_loss with a name blacklist)
        raise NotImplementedError("use_l2_regularization=True is not built (off in the configs)")
    half = hp.cbhg_out_units // 2
    assert hp.cbhg_out_units % 2 == 0
    if hp.projection2_out_channels != hp.encoder_prenet_out_units[-1]:
        raise ValueError("CBHG residual needs projection2_out_channels == prenet width "
                         "(modules/module.py:86)")
    if hp.decoder_self_attention_out_units != hp.decoder_out_units:
        raise ValueError("decoder self-attention residual needs equal widths (module.py:369)")
    if hp.self_attention_out_units % hp.self_attention_num_heads:
        raise ValueError("self_attention_out_units must divide by heads (self_attention.py:95)")
    return Dims(
        num_symbols=hp.num_symbols, embed=hp.embedding_dim,
        enc_prenet=tuple(hp.encoder_prenet_out_units), conv_ch=hp.conv_channels,
        max_k=hp.max_filter_width, proj1=hp.projection1_out_channels,
        proj2=hp.projection2_out_channels, cbhg_half=half, num_highway=hp.num_highway,
        needs_adjust=hp.projection2_out_channels != half, m1=hp.cbhg_out_units,
        m2=hp.self_attention_out_units, enc_heads=hp.self_attention_num_heads,
        enc_hops=hp.self_attention_num_hop, dec_prenet=tuple(hp.decoder_prenet_out_units),
        feed=hp.num_mels * hp.n_feed_frame, att_rnn=hp.attention_out_units,
        att1=hp.attention, att2=hp.attention2, d1=hp.attention1_out_units,
        d2=hp.attention2_out_units, loc_k=hp.attention_kernel, loc_f=hp.attention_filters,
        dec=hp.decoder_out_units, dsa=hp.decoder_self_attention_out_units,
        dec_heads=hp.decoder_self_attention_num_heads, dec_hops=hp.decoder_self_attention_num_hop,
        num_mels=hp.num_mels, r=hp.outputs_per_step,
        multi_speaker=bool(hp.use_speaker_embedding and hp.speaker_embedd_to_prenet),
        num_speakers=hp.num_speakers, spk_dim=hp.speaker_embedding_dim,
        spk_offset=hp.speaker_embedding_offset,
    )


def _dense(out: List[ParamSpec], scope: str, fan_in: int, fan_out: int, bias: bool = True,
           bias_init: str = "zeros") -> None:
    out.append(ParamSpec(f"{scope}/kernel", (fan_in, fan_out)))
    if bias:
        out.append(ParamSpec(f"{scope}/bias", (fan_out,), bias_init))


def _attention(out: List[ParamSpec], scope: str, kind: str, mem: int, query: int, units: int,
               loc_k: int, loc_f: int) -> None:
    # BahdanauAttention memory/query layers: Dense(num_units, use_bias=False)
    _dense(out, f"{scope}/memory_layer", mem, units, bias=False)
    _dense(out, f"{scope}/query_layer", query, units, bias=False)
    if kind == "forward":
        # modules/forward_attention.py:16-23 (v_a xavier, b_a zeros), :68-78 (conv + location layer)
        out.append(ParamSpec(f"{scope}/attention_variable", (units,)))
        out.append(ParamSpec(f"{scope}/attention_bias", (units,), "zeros"))
        out.append(ParamSpec(f"{scope}/location_conv/kernel", (loc_k, 1, loc_f)))
        out.append(ParamSpec(f"{scope}/location_conv/bias", (loc_f,), "zeros"))
        _dense(out, f"{scope}/location_layer", loc_f, units, bias=False)
    else:
        # TF _bahdanau_score: attention_v [num_units], no bias (normalize=False)
        out.append(ParamSpec(f"{scope}/attention_v", (units,)))


def _mha(out: List[ParamSpec], scope: str, width: int, model: int) -> None:
    # modules/self_attention.py:103-106 -- four Dense(model_dim) with bias
    for p in ("query", "key", "value"):
        _dense(out, f"{scope}/{p}_projection", width, model)
    _dense(out, f"{scope}/output_projection", model, model)


def param_specs(hp) -> List[ParamSpec]:
    d = resolve_dims(hp)
    s: List[ParamSpec] = []
    # Embedding (ext tacotron2; models/models.py:28)
    s.append(ParamSpec("embedding", (d.num_symbols, d.embed)))
    # SelfAttentionCBHGEncoder (modules/module.py:374-441)
    w = d.embed
    for i, u in enumerate(d.enc_prenet):
        _dense(s, f"encoder/prenet{i}", w, u)
        w = u
    # conv bank K=1..max_k (module.py:46-52).  Grouped by kind so the 16 BatchNorm gammas /
    # betas / biases are each ONE contiguous [max_k * C] vector: the bank's BN runs as a single
    # launch over the concatenated 2048 channels.
    bank = [f"encoder/cbhg/conv_bank/K{k}" for k in range(1, d.max_k + 1)]
    for k, sc in enumerate(bank, start=1):
        s.append(ParamSpec(f"{sc}/kernel", (k, w, d.conv_ch)))
    for sc in bank:
        s.append(ParamSpec(f"{sc}/bias", (d.conv_ch,), "zeros"))
    for sc in bank:
        s.append(ParamSpec(f"{sc}/bn/gamma", (d.conv_ch,), "ones"))
    for sc in bank:
        s.append(ParamSpec(f"{sc}/bn/beta", (d.conv_ch,), "zeros"))
    for name, cin, cout in (("proj1", d.max_k * d.conv_ch, d.proj1), ("proj2", d.proj1, d.proj2)):
        sc = f"encoder/cbhg/{name}"                                   # module.py:56-68
        s.append(ParamSpec(f"{sc}/kernel", (3, cin, cout)))
        s.append(ParamSpec(f"{sc}/bias", (cout,), "zeros"))
        s.append(ParamSpec(f"{sc}/bn/gamma", (cout,), "ones"))
        s.append(ParamSpec(f"{sc}/bn/beta", (cout,), "zeros"))
    hw = d.proj2
    if d.needs_adjust:                                                # module.py:88-89
        _dense(s, "encoder/cbhg/adjustment", d.proj2, d.cbhg_half)
        hw = d.cbhg_half
    for i in range(d.num_highway):                                    # ext HighwayNet, T bias -1
        _dense(s, f"encoder/cbhg/highway{i}/H", hw, hw)
        _dense(s, f"encoder/cbhg/highway{i}/T", hw, hw, bias_init="const:-1.0")
    for dr in ("fw", "bw"):                                           # module.py:93-108
        _dense(s, f"encoder/cbhg/lstm_{dr}", hw + d.cbhg_half, 4 * d.cbhg_half)
    _dense(s, "encoder/self_attention_projection", d.m1, d.m2)       # module.py:429
    for h in range(d.enc_hops):                                       # module.py:345-371
        _mha(s, f"encoder/self_attention{h}/mha", d.m2, d.m2)
        _dense(s, f"encoder/self_attention{h}/transform", d.m2, d.m2)
    # DualSourceTransformerDecoder (modules/module.py:1455-1562)
    if d.multi_speaker:
        s.append(ParamSpec("speaker_embedding", (d.num_speakers, d.spk_dim)))
        p0 = d.dec_prenet[0]                                          # multi_speaker_modules.py:19-21
        _dense(s, "decoder/prenet0/dense0", d.feed, p0)
        _dense(s, "decoder/prenet0/speaker_projection", d.spk_dim, p0)
        _dense(s, "decoder/prenet0/dense", p0, p0)
        w = p0
        for i, u in enumerate(d.dec_prenet[1:], start=1):
            _dense(s, f"decoder/prenet{i}", w, u)
            w = u
    else:
        w = d.feed
        for i, u in enumerate(d.dec_prenet):
            _dense(s, f"decoder/prenet{i}", w, u)
            w = u
    p_last = w
    _dense(s, "decoder/attention_lstm", p_last + d.m1 + d.m2 + d.att_rnn, 4 * d.att_rnn)
    _attention(s, "decoder/attention1", d.att1, d.m1, d.att_rnn, d.d1, d.loc_k, d.loc_f)
    _attention(s, "decoder/attention2", d.att2, d.m2, d.att_rnn, d.d2, d.loc_k, d.loc_f)
    _dense(s, "decoder/lstm1", d.att_rnn + d.m1 + d.m2 + d.dec, 4 * d.dec)
    _dense(s, "decoder/lstm2", d.dec + d.dec, 4 * d.dec)
    for h in range(d.dec_hops):                                       # module.py:700-709
        _mha(s, f"decoder/self_attention{h}/mha", d.dec, d.dsa)
        _dense(s, f"decoder/self_attention{h}/transform", d.dsa, d.dsa)
    _dense(s, "decoder/out_projection", d.dsa, d.num_mels * d.r)     # module.py:717-724
    _dense(s, "decoder/stop_token_projection", d.dsa, 1)
    return s


def bn_buffer_names(hp) -> List[Tuple[str, int]]:
    """(scope, channels) for every BatchNormalization; moving stats are non-trainable."""
    d = resolve_dims(hp)
    out = [(f"encoder/cbhg/conv_bank/K{k}/bn", d.conv_ch) for k in range(1, d.max_k + 1)]
    out += [("encoder/cbhg/proj1/bn", d.proj1), ("encoder/cbhg/proj2/bn", d.proj2)]
    return out


def _glorot(rng: np.random.Generator, shape: Tuple[int, ...]) -> np.ndarray:
    if len(shape) == 1:
        fan_in = fan_out = shape[0]
    elif len(shape) == 2:
        fan_in, fan_out = shape
    else:
        rf = int(np.prod(shape[:-2]))
        fan_in, fan_out = shape[-2] * rf, shape[-1] * rf
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape)


def init_params(hp, seed: int = 1234) -> Dict[str, np.ndarray]:
    """Seeded synthetic weights (glorot kernels, zero biases, highway T
    bias -1, BN gamma 1 / beta 0).  float32 arrays."""
    return init_specs(param_specs(hp), seed)


def init_specs(specs: List[ParamSpec], seed: int = 1234) -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(seed)
    out: Dict[str, np.ndarray] = {}
    for p in specs:
        if p.init == "glorot":
            a = _glorot(rng, p.shape)
        elif p.init == "zeros":
            a = np.zeros(p.shape)
        elif p.init == "ones":
            a = np.ones(p.shape)
        elif p.init.startswith("const:"):
            a = np.full(p.shape, float(p.init.split(":", 1)[1]))
        else:
            raise ValueError(p.init)
        out[p.name] = a.astype(np.float32)
    return out


def init_bn_buffers(hp) -> Dict[str, np.ndarray]:
    out = {}
    for scope, ch in bn_buffer_names(hp):
        out[f"{scope}/moving_mean"] = np.zeros(ch, np.float32)
        out[f"{scope}/moving_variance"] = np.ones(ch, np.float32)
    return out


LSTM_SCOPES = ("encoder/cbhg/lstm_fw", "encoder/cbhg/lstm_bw", "decoder/attention_lstm",
               "decoder/lstm1", "decoder/lstm2")


def is_lstm_param(name: str) -> bool:
    return any(name == f"{s}/kernel" or name == f"{s}/bias" for s in LSTM_SCOPES)


def to_internal(name: str, a: np.ndarray) -> np.ndarray:
    """TF LSTMCell column order [i(U) j(U) f(U) o(U)] -> gate-interleaved [U][4] (the layout the
    HIP step kernels read: one float4 per unit).  Other parameters are unchanged."""
    if not is_lstm_param(name):
        return a
    if a.ndim == 2:
        K, G = a.shape
        return a.reshape(K, 4, G // 4).transpose(0, 2, 1).reshape(K, G)
    return a.reshape(4, -1).T.reshape(-1)


def from_internal(name: str, a: np.ndarray) -> np.ndarray:
    if not is_lstm_param(name):
        return a
    if a.ndim == 2:
        K, G = a.shape
        return a.reshape(K, G // 4, 4).transpose(0, 2, 1).reshape(K, G)
    return a.reshape(-1, 4).T.reshape(-1)


class Layout:
    """Offsets of every parameter inside one flat fp32 arena (256-byte aligned)."""

    def __init__(self, specs: List[ParamSpec]):
        self.specs = list(specs)
        self.offsets: Dict[str, int] = {}
        self.shapes: Dict[str, Tuple[int, ...]] = {}
        off = 0
        for p in self.specs:
            off = (off + ALIGN_FLOATS - 1) // ALIGN_FLOATS * ALIGN_FLOATS
            self.offsets[p.name] = off
            self.shapes[p.name] = p.shape
            off += int(np.prod(p.shape))
        self.total = (off + ALIGN_FLOATS - 1) // ALIGN_FLOATS * ALIGN_FLOATS
        self.num_params = sum(int(np.prod(p.shape)) for p in self.specs)

    def pack(self, values: Dict[str, np.ndarray], internal: bool = True) -> np.ndarray:
        """TF-layout arrays -> flat arena (LSTM tensors gate-interleaved when internal)."""
        flat = np.zeros(self.total, np.float32)
        for p in self.specs:
            o = self.offsets[p.name]
            a = np.asarray(values[p.name], np.float32).reshape(p.shape)
            if internal:
                a = to_internal(p.name, a)
            flat[o:o + int(np.prod(p.shape))] = a.ravel()
        return flat

    def unpack(self, flat: np.ndarray, internal: bool = True) -> Dict[str, np.ndarray]:
        """flat arena -> TF-layout arrays (inverse of pack)."""
        out = {}
        for p in self.specs:
            o = self.offsets[p.name]
            a = np.asarray(flat[o:o + int(np.prod(p.shape))]).reshape(p.shape)
            out[p.name] = from_internal(p.name, a) if internal else a
        return out

    def views(self, arena) -> Dict[str, "object"]:
        """Name -> view into a torch (or numpy) 1-D arena."""
        return {p.name: arena[self.offsets[p.name]:self.offsets[p.name] + int(np.prod(p.shape))]
                .view(*p.shape) if hasattr(arena, "view") and not isinstance(arena, np.ndarray)
                else arena[self.offsets[p.name]:self.offsets[p.name] + int(np.prod(p.shape))]
                .reshape(p.shape) for p in self.specs}


def count_params(hp) -> int:
    return sum(int(np.prod(p.shape)) for p in param_specs(hp))


def maybe(d: Dict[str, np.ndarray], name: str) -> Optional[np.ndarray]:
    return d.get(name)
