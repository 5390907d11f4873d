"""Attention plugin surface: ``AttentionOptions`` + ``attention_mechanism_factory``.

Mirrors modules/attentions.py:15-62 (the factory keyed by ``options.attention``) and
models/attention_factories.py:11-37 (``attention_factory`` / ``dual_source_attention_factory``
building options from hparams).  ``attention_fn(memory, memory_sequence_length,
teacher_alignments=None)`` returns a mechanism object with the TF ``AttentionMechanism``
protocol the reference relies on (modules/forward_attention.py:88-136): ``keys``, ``values``,
``alignments_size``, ``state_size``, ``initial_alignments(batch_size, dtype)``,
``initial_state(batch_size, dtype)`` and ``__call__(query, state) -> (alignments, next_state)``.

The mechanisms are HIP-backed: memory masking and the memory layer run on libsat_hip at
construction, and every ``__call__`` runs one attention step through ``sat_attn_step_fwd`` (the
dual-source tile kernel, with this mechanism as source 1).  Inside the decoder the two
mechanisms of ``dual_source_attention_factory`` are fused into ONE kernel per step; the
per-mechanism call here is the plugin-level entry for stepping a single mechanism.

Supported kinds on this path: ``"forward"`` (ForwardAttention), ``"additive"``
(BahdanauAttention) and the forced-alignment kinds ``"teacher_forcing_forward"`` /
``"teacher_forcing_additive"`` (modules/teacher_forcing_attention.py:13-78: step ``index``
returns ``teacher_alignments[:, index]``; used by ``force_alignment_*_factory`` and the
``use_forced_alignment_mode`` pass of model_fn).  ``"location_sensitive"`` is a reference kind
outside the LJSpeech/VCTK self-attention configs: it raises ``NotImplementedError``; unknown
kinds raise ``ValueError`` like the reference.
"""

from __future__ import annotations

from collections import namedtuple
from typing import Dict, Optional

import torch

from . import kernels as K
from . import params as PR


class AttentionOptions(namedtuple("AttentionOptions", ["attention",
                                                       "num_units",
                                                       "attention_kernel",
                                                       "attention_filters",
                                                       "smoothing",
                                                       "cumulative_weights",
                                                       "use_transition_agent"])):
    pass


_OUT_OF_SCOPE = ("location_sensitive",)
_DUMMY_D2, _DUMMY_M2 = 32, 4     # inert second source when a single mechanism is stepped


class _HipAttention:
    """Shared part of the HIP-backed mechanisms: memory preparation (TF _prepare_memory:
    values = memory masked past memory_sequence_length; keys = memory_layer(values))."""

    kind = ""

    def __init__(self, options: AttentionOptions, memory: torch.Tensor,
                 memory_sequence_length: torch.Tensor, variables: Optional[Dict] = None,
                 query_depth: Optional[int] = None, seed: int = 1234):
        if memory.dtype != torch.float32 or not memory.is_cuda:
            raise TypeError("memory must be a float32 device tensor [B, N, M]")
        if options.cumulative_weights:
            raise NotImplementedError("cumulative_weights=True is not on the hot path")
        if options.use_transition_agent:
            raise NotImplementedError("use_transition_agent=True is not on the hot path")
        self.options = options
        self.B, self.N, self.M = memory.shape
        self.lengths = memory_sequence_length.to(device=memory.device, dtype=torch.int64)
        self.units = int(options.num_units)
        self.query_depth = query_depth
        if variables is None:
            if query_depth is None:
                raise ValueError("query_depth is needed to create the mechanism's variables")
            specs = []
            PR._attention(specs, "m", self.kind, self.M, query_depth, self.units,
                          int(options.attention_kernel), int(options.attention_filters))
            vals = PR.init_specs(specs, seed)
            variables = {k[2:]: torch.tensor(v, device=memory.device) for k, v in vals.items()}
        self.variables = variables
        self.values = K.seq_mask(memory.contiguous(), self.lengths)
        self.keys = K.linear(self.values, variables["memory_layer/kernel"])
        self._scratch = None

    # ---- TF AttentionMechanism protocol
    @property
    def alignments_size(self) -> int:
        return self.N

    @property
    def state_size(self) -> int:
        return self.N

    def initial_alignments(self, batch_size: int, dtype=torch.float32) -> torch.Tensor:
        return torch.zeros(batch_size, self.N, dtype=dtype, device=self.values.device)

    # ---- one step through the tile kernel
    def _step(self, query: torch.Tensor, s_prev, a_prev):
        B, N, dev = self.B, self.N, self.values.device
        f32 = dict(device=dev, dtype=torch.float32)
        if self._scratch is None:
            ntiles = (N + 31) // 32
            pst = K.part_stride(self.M, _DUMMY_M2)
            self._scratch = dict(
                ntiles=ntiles, pst=pst, e1=torch.empty(B, N, **f32), e2=torch.empty(B, N, **f32),
                part=torch.empty(B, ntiles, pst, **f32),
                K2=torch.zeros(B, N, _DUMMY_D2, **f32), V2=torch.zeros(B, N, _DUMMY_M2, **f32),
                v2=torch.zeros(_DUMMY_D2, **f32))
        sc = self._scratch
        v = self.variables
        q = torch.zeros(B, self.units + _DUMMY_D2, **f32)
        K.gemm(query.contiguous(), v["query_layer/kernel"], q[:, :self.units])
        s_out, a_out, s2 = (torch.empty(B, N, **f32) for _ in range(3))
        ctx = torch.empty(B, self.M + _DUMMY_M2, **f32)
        fwd = self.kind == "forward"
        K.attn_step_fwd(
            B=B, N=N, D1=self.units, M1=self.M, D2=_DUMMY_D2, M2=_DUMMY_M2,
            F=int(self.options.attention_filters), KW=int(self.options.attention_kernel), NT=32,
            ntiles=sc["ntiles"], att1_forward=1 if fwd else 0, u=0.5, q=q,
            q_sb=self.units + _DUMMY_D2, K1=self.keys, V1=self.values, K2=sc["K2"], V2=sc["V2"],
            lengths=self.lengths, s_prev=s_prev, a_prev=a_prev,
            v1=v["attention_variable"] if fwd else v["attention_v"],
            b1=v["attention_bias"] if fwd else None,
            convW=v["location_conv/kernel"] if fwd else None,
            convb=v["location_conv/bias"] if fwd else None,
            locW=v["location_layer/kernel"] if fwd else None, v2=sc["v2"], e1=sc["e1"],
            e2=sc["e2"], part=sc["part"], part_stride=sc["pst"], s_out=s_out, a_out=a_out,
            s2_out=s2, ctx=ctx, ctx_sb=self.M + _DUMMY_M2, stats=None)
        return s_out, a_out, ctx[:, :self.M]


class ForwardAttention(_HipAttention):
    """modules/forward_attention.py:48-136 (ForwardAttention, no transition agent, no
    cumulative weights).  state = (s_{t-1}, alpha_{t-1}, u)."""

    kind = "forward"

    def initial_state(self, batch_size: int, dtype=torch.float32):     # :128-136
        dev = self.values.device
        s0 = torch.zeros(batch_size, self.N, dtype=dtype, device=dev)
        a0 = torch.zeros(batch_size, self.N, dtype=dtype, device=dev)
        a0[:, 0] = 1.0
        u0 = torch.full((batch_size, 1), 0.5, dtype=dtype, device=dev)
        return s0, a0, u0

    def __call__(self, query, state):                                   # :88-122
        s_prev, a_prev, u = state
        s, a, _ = self._step(query, s_prev.contiguous(), a_prev.contiguous())
        return a, (s, a, u)


class BahdanauAttention(_HipAttention):
    """TF contrib BahdanauAttention(num_units, normalize=False) as built at
    modules/attentions.py:53-57.  state = previous alignments (unused by the score)."""

    kind = "additive"

    def initial_state(self, batch_size: int, dtype=torch.float32):
        return self.initial_alignments(batch_size, dtype)

    def __call__(self, query, state):
        s, _, _ = self._step(query, None, None)
        return s, s


class TeacherForcingAttention:
    """TeacherForcingForwardAttention / TeacherForcingAdditiveAttention
    (modules/teacher_forcing_attention.py:13-78).  Memory preparation is TF BahdanauAttention's
    (values = memory masked past memory_sequence_length, on libsat_hip); the memory layer's keys
    are never read by ``__call__`` and are not formed.  State = (previous alignments, index),
    initial index -1 (:38-41); ``__call__`` ignores the query and returns
    ``teacher_alignments[:, index + 1]`` as both the alignments and the next state's alignments
    (:30-35).  ``teacher_alignments``: [B, T', N] device tensor."""

    def __init__(self, kind: str, options: AttentionOptions, memory: torch.Tensor,
                 memory_sequence_length: torch.Tensor, teacher_alignments: torch.Tensor):
        if memory.dtype != torch.float32 or not memory.is_cuda:
            raise TypeError("memory must be a float32 device tensor [B, N, M]")
        if teacher_alignments is None:
            raise ValueError(f"{kind} attention needs teacher_alignments [B, T', N]")
        B, N, _ = memory.shape
        if (teacher_alignments.dim() != 3 or teacher_alignments.shape[0] != B
                or teacher_alignments.shape[2] != N):
            raise ValueError(f"teacher_alignments must be [B={B}, T', N={N}], got "
                             f"{tuple(teacher_alignments.shape)}")
        self.kind = kind
        self.options = options
        self.batch_size, self.N = B, N
        self.values = K.seq_mask(memory.contiguous(), memory_sequence_length)
        self.teacher_alignments = teacher_alignments

    @property
    def alignments_size(self) -> int:
        return self.N

    @property
    def state_size(self):
        return self.N, 1

    def initial_alignments(self, batch_size: int, dtype=torch.float32) -> torch.Tensor:
        return torch.zeros(batch_size, self.N, device=self.values.device, dtype=dtype)

    def initial_state(self, batch_size: int, dtype=torch.float32):
        return self.initial_alignments(batch_size, dtype), -1

    def __call__(self, query, state):
        _, prev_index = state
        index = int(prev_index) + 1
        alignments = self.teacher_alignments[:, index]
        return alignments, (alignments, index)


def attention_mechanism_factory(options: AttentionOptions):
    """modules/attentions.py:25-62."""
    def attention_fn(memory, memory_sequence_length, teacher_alignments=None, variables=None,
                     query_depth=None, seed=1234):
        if options.attention == "forward":
            cls = ForwardAttention
        elif options.attention == "additive":
            cls = BahdanauAttention
        elif options.attention in ("teacher_forcing_forward", "teacher_forcing_additive"):
            return TeacherForcingAttention(options.attention, options, memory,
                                           memory_sequence_length, teacher_alignments)
        elif options.attention in _OUT_OF_SCOPE:
            raise NotImplementedError(
                f"attention mechanism {options.attention!r} is outside the hot path "
                "(LJSpeech/VCTK self-attention configs use 'forward' + 'additive')")
        else:
            raise ValueError(f"Unknown attention mechanism: {options.attention}")
        return cls(options, memory, memory_sequence_length, variables=variables,
                   query_depth=query_depth, seed=seed)

    attention_fn.options = options
    return attention_fn


def attention_factory(params):
    """models/attention_factories.py:11-19."""
    return attention_mechanism_factory(AttentionOptions(
        attention=params.attention, num_units=params.attention_out_units,
        attention_kernel=params.attention_kernel, attention_filters=params.attention_filters,
        smoothing=False, cumulative_weights=params.cumulative_weights,
        use_transition_agent=params.use_forward_attention_transition_agent))


def dual_source_attention_factory(params):
    """models/attention_factories.py:22-37."""
    common = dict(attention_kernel=params.attention_kernel,
                  attention_filters=params.attention_filters, smoothing=False,
                  cumulative_weights=params.cumulative_weights,
                  use_transition_agent=params.use_forward_attention_transition_agent)
    o1 = AttentionOptions(attention=params.attention, num_units=params.attention1_out_units,
                          **common)
    o2 = AttentionOptions(attention=params.attention2, num_units=params.attention2_out_units,
                          **common)
    return attention_mechanism_factory(o1), attention_mechanism_factory(o2)


def force_alignment_attention_factory(params):
    """models/attention_factories.py:40-48."""
    return attention_mechanism_factory(AttentionOptions(
        attention=params.forced_alignment_attention, num_units=params.attention_out_units,
        attention_kernel=params.attention_kernel, attention_filters=params.attention_filters,
        smoothing=False, cumulative_weights=params.cumulative_weights,
        use_transition_agent=params.use_forward_attention_transition_agent))


def force_alignment_dual_source_attention_factory(params):
    """models/attention_factories.py:51-66."""
    common = dict(attention_kernel=params.attention_kernel,
                  attention_filters=params.attention_filters, smoothing=False,
                  cumulative_weights=params.cumulative_weights,
                  use_transition_agent=params.use_forward_attention_transition_agent)
    o1 = AttentionOptions(attention=params.forced_alignment_attention,
                          num_units=params.attention1_out_units, **common)
    o2 = AttentionOptions(attention=params.forced_alignment_attention2,
                          num_units=params.attention2_out_units, **common)
    return attention_mechanism_factory(o1), attention_mechanism_factory(o2)


def mechanism_variables(P: Dict[str, torch.Tensor], scope: str) -> Dict[str, torch.Tensor]:
    """The scope-relative variables of one mechanism from the model's parameter views."""
    pre = scope.rstrip("/") + "/"
    return {k[len(pre):]: v for k, v in P.items() if k.startswith(pre)}


__all__ = ["AttentionOptions", "attention_mechanism_factory", "attention_factory",
           "dual_source_attention_factory", "force_alignment_attention_factory",
           "force_alignment_dual_source_attention_factory", "TeacherForcingAttention",
           "ForwardAttention", "BahdanauAttention",
           "mechanism_variables"]
