"""ctypes binding of ``libsat_hip.so`` (declared in ``include/sat_abi.h``).

Torch tensors are plumbing: only their device pointers, sizes and the current HIP stream cross
the boundary.  There is no fallback -- if the library is missing or was not built for this GPU,
every op raises ``SatLibraryError``.
"""

from __future__ import annotations

import ctypes
import os
from typing import Optional

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# SAT_LIB_OVERRIDE: an instrumented build for the probes under tools/ (never set by the product)
LIB_PATH = os.environ.get("SAT_LIB_OVERRIDE") or os.path.join(PKG_DIR, "libsat_hip.so")


class SatLibraryError(RuntimeError):
    """A library call failed; ``rc`` is its SAT_ERR_* code (None when raised host-side)."""

    def __init__(self, msg: str, rc: Optional[int] = None):
        super().__init__(msg)
        self.rc = rc


SAT_ERR_UNSUPPORTED = -3


class SatGemmDesc(ctypes.Structure):
    _fields_ = [
        ("M", ctypes.c_int32), ("N", ctypes.c_int32), ("K", ctypes.c_int32),
        ("batch", ctypes.c_int32),
        ("a_mode", ctypes.c_int32), ("a_L", ctypes.c_int32), ("a_C", ctypes.c_int32),
        ("a_shift", ctypes.c_int32),
        ("A", ctypes.c_void_p),
        ("a_sm", ctypes.c_int64), ("a_sk", ctypes.c_int64), ("a_sbatch", ctypes.c_int64),
        ("b_mode", ctypes.c_int32), ("b_taps", ctypes.c_int32), ("b_C", ctypes.c_int32),
        ("act", ctypes.c_int32),
        ("B", ctypes.c_void_p),
        ("b_sk", ctypes.c_int64), ("b_sn", ctypes.c_int64), ("b_sbatch", ctypes.c_int64),
        ("C", ctypes.c_void_p),
        ("c_sm", ctypes.c_int64), ("c_sbatch", ctypes.c_int64),
        ("bias", ctypes.c_void_p), ("bias_sbatch", ctypes.c_int64),
        ("alpha", ctypes.c_float), ("beta", ctypes.c_float),
        ("mul", ctypes.c_void_p), ("mul_sm", ctypes.c_int64), ("mul_sbatch", ctypes.c_int64),
        ("batch2", ctypes.c_int32), ("tri", ctypes.c_int32),
        ("a_sbatch2", ctypes.c_int64), ("b_sbatch2", ctypes.c_int64),
        ("c_sbatch2", ctypes.c_int64), ("mul_sbatch2", ctypes.c_int64),
        ("add", ctypes.c_void_p), ("add_sm", ctypes.c_int64), ("add_sbatch", ctypes.c_int64),
        ("ws", ctypes.c_void_p), ("ws_bytes", ctypes.c_int64),
        ("colsum_out", ctypes.c_void_p),
        ("A2", ctypes.c_void_p),
        ("a2_sm", ctypes.c_int64),
        ("k1", ctypes.c_int32),
        ("pad1", ctypes.c_int32),
        ("C2", ctypes.c_void_p),
        ("c2_sm", ctypes.c_int64),
        ("n1", ctypes.c_int32),
        ("pad2", ctypes.c_int32),
        ("B2", ctypes.c_void_p),
        ("b2_s", ctypes.c_int64),
    ]


_P = ctypes.c_void_p
_I32, _I64, _U64, _F = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float


def _struct(name, spec):
    """spec: 'type:field ...' with types i32 i64 f32 ptr."""
    tmap = {"i32": _I32, "i64": _I64, "f32": _F, "ptr": _P}
    fields = [(f, tmap[t]) for t, f in (item.split(":") for item in spec.split())]
    return type(name, (ctypes.Structure,), {"_fields_": fields})


SatLstmFwd = _struct("SatLstmFwd", """
    i32:B i32:U i32:K i32:t ptr:xproj i64:xproj_sb ptr:bias ptr:rin i64:rin_sb ptr:W
    ptr:c_prev ptr:h_prev i64:h_prev_sb ptr:mask_c ptr:mask_h f32:zc f32:zh ptr:lengths
    ptr:h_raw i64:h_raw_sb ptr:c_out ptr:h_out i64:h_out_sb ptr:gates
    ptr:rin1 i64:rin1_sb ptr:rin2 i64:rin2_sb i32:K1 i32:K2""")

SatLstmBwd = _struct("SatLstmBwd", """
    i32:B i32:U i32:K i32:hoff i32:t ptr:W ptr:dgates_next ptr:gates ptr:c_prev
    ptr:dy i64:dy_sb ptr:dq0 ptr:wq0 i32:dq0_n ptr:dq1 ptr:wq1 i32:dq1_n
    i32:dq_parts i64:dq_pstride i64:dq_bstride ptr:dh_carry ptr:dc_carry ptr:mask_c ptr:mask_h f32:zc f32:zh ptr:lengths
    ptr:dgates ptr:dh_carry_out ptr:dc_carry_out ptr:rec i64:rec_sb""")

SatConvBank = _struct("SatConvBank", """
    i32:S i32:L i32:C i32:max_k i32:Co i32:pad0 ptr:x i64:x_sm ptr:W ptr:bias ptr:y i64:y_sm
    ptr:dx i64:dx_sm ptr:dW f32:beta_dx f32:beta_dw ptr:ws i64:ws_bytes""")

SatMha = _struct("SatMha", """
    i32:B i32:L i32:W i32:D i32:H i32:causal i32:out_dim i32:pad0 ptr:x ptr:Wq ptr:bq ptr:Wk
    ptr:bk ptr:Wv ptr:bv ptr:Wo ptr:bo ptr:probs_mask ptr:q ptr:k ptr:v ptr:P ptr:Pd ptr:o ptr:y
    ptr:dy ptr:dx ptr:dWq ptr:dbq ptr:dWk ptr:dbk ptr:dWv ptr:dbv ptr:dWo ptr:dbo ptr:scratch
    i64:scratch_bytes ptr:gemm_ws i64:gemm_ws_bytes ptr:lse""")

SatFlashAttn = _struct("SatFlashAttn", """
    i32:B i32:H i32:L i32:dh i32:causal f32:scale i64:ld ptr:q ptr:k ptr:v ptr:mask ptr:o ptr:lse
    ptr:dout ptr:delta ptr:dq ptr:dk ptr:dv""")

class SatRngSegment(ctypes.Structure):      # mirrors include/sat_abi.h
    _fields_ = [("offset", ctypes.c_int64), ("n", ctypes.c_int64), ("stream_id", ctypes.c_uint64),
                ("keep", ctypes.c_float), ("on_value", ctypes.c_float)]


class SatColSegment(ctypes.Structure):      # mirrors include/sat_abi.h
    _fields_ = [("dst", ctypes.c_void_p), ("col", ctypes.c_int32), ("n", ctypes.c_int32)]


SatDims = _struct("SatDims", """
    i32:B i32:N i32:Tp i32:enc_heads i32:dec_heads i32:enc_D i32:dec_D i32:max_cols""")

SatAdamConfig = _struct("SatAdamConfig", """
    f32:lr0 f32:beta1 f32:beta2 f32:eps f32:clip_norm i32:decay i32:step_factor f32:grad_scale""")

SatAttnStepBwd = _struct("SatAttnStepBwd", """
    i32:B i32:N i32:D1 i32:M1 i32:D2 i32:M2 i32:F i32:KW i32:NT i32:ntiles i32:att1_forward
    f32:u ptr:dctx i64:dctx_sb ptr:ctx_t i64:ctx_sb ptr:y_next ptr:V1 ptr:V2 ptr:s_t ptr:a_t
    ptr:a_prev ptr:s_prev ptr:s2_t ptr:stats ptr:df_next ptr:q i64:q_sb ptr:K1 ptr:K2
    ptr:v1 ptr:b1 ptr:convW ptr:convb ptr:locW ptr:v2 ptr:y_out ptr:df_out ptr:de1_out ptr:de2_out
    ptr:dqp i32:waves""")

SatAttnParamGrad = _struct("SatAttnParamGrad", """
    i32:T i32:B i32:N i32:D1 i32:D2 i32:F i32:KW i32:att1_forward ptr:K1 ptr:K2
    ptr:q i64:q_tstride i64:q_bstride ptr:b1 ptr:v1 ptr:locW ptr:v2 ptr:loc
    ptr:s_prev i64:s_tstride ptr:de1 ptr:de2 ptr:df ptr:dK1 ptr:dK2 ptr:pg i64:pg_stride
    i32:tsplit""")

SatDecAttnFwd = _struct("SatDecAttnFwd", """
    i32:B i32:N i32:T i32:U i32:M1 i32:M2 i32:D1 i32:D2 i32:F i32:KW f32:u f32:zc f32:zh
    ptr:X0 ptr:W0r ptr:Wq1 ptr:Wq2 ptr:K1 ptr:V1 ptr:K2 ptr:V2 ptr:lengths
    ptr:v1 ptr:b1 ptr:convW ptr:convb ptr:locW ptr:v2 ptr:mask_c ptr:mask_h
    ptr:REC0 ptr:C0 ptr:H0RAW ptr:G0 ptr:Q ptr:S1 ptr:AL1 ptr:S2 ptr:ST ptr:LOC
    ptr:E ptr:PART ptr:QP ptr:ctr ptr:err ptr:prof ptr:ZH""")

SatDecAttnBwd = _struct("SatDecAttnBwd", """
    i32:B i32:N i32:T i32:U i32:M1 i32:M2 i32:D1 i32:D2 i32:F i32:KW f32:u f32:zc f32:zh
    ptr:REC0 ptr:C0 ptr:G0 ptr:S1 ptr:AL1 ptr:S2 ptr:ST ptr:LOC
    ptr:V1 ptr:V2 ptr:v1 ptr:convW ptr:convb ptr:locW ptr:v2
    ptr:W0r ptr:Wq1 ptr:Wq2 ptr:mask_c ptr:mask_h ptr:DH0 ptr:ZH
    ptr:RD ptr:DG0 ptr:DE1 ptr:DE2 ptr:DFH ptr:DQP ptr:RDP ptr:YA ptr:ctr ptr:err ptr:prof""")

SatDecLstmFwd = _struct("SatDecLstmFwd", """
    i32:B i32:T i32:U f32:zc f32:zh ptr:X1 ptr:W1r ptr:W2 ptr:b2
    ptr:mask1_c ptr:mask1_h ptr:mask2_c ptr:mask2_h
    ptr:H1RAW ptr:C1S ptr:H1S ptr:G1 ptr:H2RAW ptr:C2S ptr:H2S ptr:G2 ptr:xch ptr:err ptr:prof""")

SatDecLstmBwd = _struct("SatDecLstmBwd", """
    i32:B i32:T i32:U f32:zc f32:zh ptr:W1r ptr:W2 ptr:G1 ptr:C1S ptr:G2 ptr:C2S ptr:DH2
    ptr:mask1_c ptr:mask1_h ptr:mask2_c ptr:mask2_h ptr:DG1 ptr:DG2 ptr:ctr ptr:err ptr:prof""")

SatDecodePersistent = _struct("SatDecodePersistent", """
    i32:B i32:N i32:T i32:min_iters i32:stop_mode f32:zc f32:zh f32:u f32:scale
    ptr:lengths ptr:K1 ptr:V1 ptr:K2 ptr:V2 ptr:Wzp ptr:bzp ptr:bp0 ptr:Wp1 ptr:bp1 ptr:W0 ptr:b0
    ptr:Wq ptr:b1 ptr:v1 ptr:convW ptr:convb ptr:locW ptr:v2 ptr:W1 ptr:bl1 ptr:W2 ptr:bl2
    ptr:Wqku ptr:bqku ptr:bz ptr:Wms ptr:bms ptr:MS ptr:AL1 ptr:S2 ptr:SA_P ptr:state
    ptr:scratch i64:scratch_bytes ptr:err ptr:prof""")


class SatDecoderLoopFwd(ctypes.Structure):   # mirrors include/sat_abi.h
    _fields_ = [("attn", SatDecAttnFwd), ("lstm", SatDecLstmFwd), ("W1x", _P), ("b1", _P),
                ("ws", _P), ("ws_bytes", _I64)]


class SatDecoderLoopBwd(ctypes.Structure):   # mirrors include/sat_abi.h
    _fields_ = [("lstm", SatDecLstmBwd), ("attn", SatDecAttnBwd), ("W1x", _P), ("DH0", _P),
                ("ws", _P), ("ws_bytes", _I64)]


SatEncLstmFwd = _struct("SatEncLstmFwd", """
    i32:B i32:N i32:U f32:zc f32:zh ptr:X_fw ptr:X_bw i64:x_sb i64:x_sn ptr:W_fw ptr:W_bw
    ptr:mc_fw ptr:mh_fw ptr:mc_bw ptr:mh_bw ptr:lengths ptr:H i64:h_sb i64:h_sn
    ptr:CS_fw ptr:HS_fw ptr:CS_bw ptr:HS_bw ptr:G_fw ptr:G_bw""")

SatEncLstmBwd = _struct("SatEncLstmBwd", """
    i32:B i32:N i32:U f32:zc f32:zh ptr:W_fw ptr:W_bw ptr:G_fw ptr:G_bw ptr:CS_fw ptr:CS_bw
    ptr:mc_fw ptr:mh_fw ptr:mc_bw ptr:mh_bw ptr:lengths ptr:DY i64:dy_sb i64:dy_sn
    ptr:DG_fw ptr:DG_bw""")

SatAttnStep = _struct("SatAttnStep", """
    i32:B i32:N i32:D1 i32:M1 i32:D2 i32:M2 i32:F i32:KW i32:NT i32:ntiles i32:att1_forward
    f32:u ptr:q i64:q_sb ptr:K1 ptr:V1 ptr:K2 ptr:V2 ptr:lengths ptr:s_prev ptr:a_prev
    ptr:v1 ptr:b1 ptr:convW ptr:convb ptr:locW ptr:v2 ptr:e1 ptr:e2 ptr:part i64:part_stride
    ptr:s_out ptr:a_out ptr:s2_out ptr:ctx i64:ctx_sb ptr:stats ptr:loc_out i32:lpp i32:phases""")

# name -> argtypes (restype is int for all but sat_last_error_string)
SIGNATURES = {
    "sat_version": [],
    "sat_abi_version": [],
    "sat_device_arch": [ctypes.c_char_p, _I32],
    "sat_gemm": [ctypes.POINTER(SatGemmDesc), _P],
    "sat_gemm_force_plan": [_I32, _I32, _I32],
    "sat_gemm_probe_mode": [_I32],
    "sat_cbhg_convbank_fwd": [ctypes.POINTER(SatConvBank), _P],
    "sat_mha_fwd": [ctypes.POINTER(SatMha), _P],
    "sat_mha_bwd": [ctypes.POINTER(SatMha), _P],
    "sat_mha_bwd_wgrad": [ctypes.POINTER(SatMha), _P],
    "sat_flash_attn_fwd": [ctypes.POINTER(SatFlashAttn), _P],
    "sat_flash_attn_bwd": [ctypes.POINTER(SatFlashAttn), _P],
    "sat_cbhg_convbank_bwd": [ctypes.POINTER(SatConvBank), _P],
    "sat_rng_fill": [_P, _I64, _P, _U64, _F, _F, _P],
    "sat_rng_fill_segments": [_P, ctypes.POINTER(SatRngSegment), _I32, _P, _P],
    "sat_counter_add": [_P, _U64, _P],
    "sat_stop_check": [_P, _I64, _I32, _I32, _I32, _P, _P],
    "sat_lstm_step_fwd": [ctypes.POINTER(SatLstmFwd), _P],
    "sat_lstm_step_bwd": [ctypes.POINTER(SatLstmBwd), _P],
    "sat_lstm_steps_fwd": [ctypes.POINTER(SatLstmFwd), _I32, _P],
    "sat_lstm_steps_bwd": [ctypes.POINTER(SatLstmBwd), _I32, _P],
    "sat_attn_part_stride": [_I32, _I32],
    "sat_attn_query": [_I32, _I32, _I32, _I32, _P, _I64, _P, _P, _P, _I64, _P],
    "sat_attn_step_fwd": [ctypes.POINTER(SatAttnStep), _P],
    "sat_attn_pg_stride": [_I32, _I32, _I32, _I32],
    "sat_attn_step_bwd": [ctypes.POINTER(SatAttnStepBwd), _P],
    "sat_decoder_attention_fwd": [ctypes.POINTER(SatDecAttnFwd), _P],
    "sat_decoder_attention_bwd": [ctypes.POINTER(SatDecAttnBwd), _P],
    "sat_decoder_lstms_fwd": [ctypes.POINTER(SatDecLstmFwd), _P],
    "sat_encoder_lstm_fwd": [ctypes.POINTER(SatEncLstmFwd), _P],
    "sat_encoder_lstm_bwd": [ctypes.POINTER(SatEncLstmBwd), _P],
    "sat_decoder_lstms_bwd": [ctypes.POINTER(SatDecLstmBwd), _P],
    "sat_decoder_loop_fwd": [ctypes.POINTER(SatDecoderLoopFwd), _P],
    "sat_decoder_loop_bwd": [ctypes.POINTER(SatDecoderLoopBwd), _P],
    "sat_decode_attention_step": [_P, _I64, _I64, _I32, _I32, _I32, _I32, _F, _P, _I32, _P,
                                  _I64, _P],
    "sat_decode_persistent": [ctypes.POINTER(SatDecodePersistent), _P],
    "sat_zlstm_step_fwd": [ctypes.POINTER(SatLstmFwd), _P],
    "sat_zlstm_step_bwd": [ctypes.POINTER(SatLstmBwd), _P],
    "sat_attn_param_grad_rows": [_I32, _I32],
    "sat_attn_param_grads": [ctypes.POINTER(SatAttnParamGrad), _P],
    "sat_seq_mask": [_P, _P, _I32, _I32, _I32, _P, _P],
    "sat_embedding_fwd": [_P, _P, _P, _I64, _I32, _I32, _I64, _P, _P],
    "sat_embedding_bwd": [_P, _P, _P, _I64, _I32, _I32, _I64, _P],
    "sat_bn_stats": [_P, _I64, _I32, _I32, _P, _P, _P, _P, _F, _P, _P],
    "sat_bn_apply": [_P, _I64, _P, _I64, _I32, _I32, _P, _P, _F, _P, _P, _I32, _P, _I64, _P],
    "sat_bn_bwd": [_P, _I64, _P, _I64, _P, _I64, _P, _I64, _I32, _I32, _P, _P, _F, _P, _P, _P,
                   _I32, _F, _P, _P],
    "sat_colsum": [_P, _I64, _I32, _I32, _P, _F, _P, _P],
    "sat_colsum_scatter": [_P, _I64, _I32, _I32, ctypes.POINTER(SatColSegment), _I32, _F, _P,
                           _P],
    "sat_maxpool2": [_P, _P, _I32, _I32, _I32, _P],
    "sat_bn_apply_maxpool2": [_P, _P, _P, _I32, _I32, _I32, _P, _P, _F, _P, _P, _I32, _P],
    "sat_maxpool2_bwd": [_P, _P, _P, _I32, _I32, _I32, _P],
    "sat_highway_fwd": [_P, _P, _P, _P, _I64, _P],
    "sat_highway_act_fwd": [_P, _P, _P, _P, _I64, _P],
    "sat_highway_bwd": [_P, _P, _P, _P, _P, _P, _P, _I64, _P],
    "sat_act_bwd": [_P, _P, _P, _P, _I64, _I32, _F, _P],
    "sat_axpby": [_P, _P, _I64, _F, _F, _P],
    "sat_fill32": [_P, _I64, ctypes.c_uint32, _P],
    "sat_add": [_P, _P, _P, _I64, _P],
    "sat_copy3d": [_P, _I64, _I64, _P, _I64, _I64, _I32, _I32, _I32, _P],
    "sat_softmax_fwd": [_P, _P, _P, _P, _I64, _I32, _I32, _I32, _F, _P],
    "sat_softmax_bwd": [_P, _P, _P, _P, _I64, _I32, _I32, _I32, _F, _P],
    "sat_loss_fwd_bwd": [_P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _F, _P, _P, _P, _P, _P],
}

SIGNATURES.update({
    "sat_transpose": [_P, _I64, _P, _I64, _I32, _I32, _P],
    "sat_gemm_rowdot": [_I32, _I32, _I32, _P, _I64, _P, _I64, _P, _I64, _F, _F, _P],
    "sat_global_norm_sq": [_P, _I64, _P, _P],
    "sat_adam_step": [_P, _P, _P, _P, _I64, _P, _P, _P, ctypes.POINTER(SatAdamConfig), _P, _I32,
                      _P, _P],
    "sat_exchange_pack": [_P, _I32, _P, _I64, _P, _F, _P],
    "sat_exchange_unpack": [_P, _I32, _P, _P],
})

RESTYPES = {"sat_workspace_colreduce": (ctypes.c_int64, [_I32, _I32]),
            "sat_workspace_adam": (ctypes.c_int64, []),
            "sat_workspace_loss": (ctypes.c_int64, []),
            "sat_mha_scratch_bytes": (ctypes.c_int64, [_I32, _I32, _I32, _I32, _I32]),
            "sat_mha_scratch_bytes_fused": (ctypes.c_int64, [_I32, _I32, _I32, _I32, _I32]),
            "sat_workspace_size": (ctypes.c_int64, [ctypes.c_void_p]),
            "sat_decoder_attention_scratch": (ctypes.c_int64, [_I32, _I32, _P, _P, _P]),
            "sat_decoder_attention_bwd_scratch": (ctypes.c_int64, [_I32, _I32, _P, _P]),
            "sat_decoder_attention_bwd_dq_parts": (ctypes.c_int32, [_I32, _I32]),
            "sat_decoder_lstms_scratch": (ctypes.c_int64, [_I32]),
            "sat_decode_persistent_scratch_bytes": (ctypes.c_int64, []),
            "sat_decoder_lstms_bwd_scratch": (ctypes.c_int64, [_I32]),
            "sat_crc32c": (ctypes.c_uint32, [_P, _I64, ctypes.c_uint32]),
            "sat_tfrecord_masked_crc": (ctypes.c_uint32, [_P, _I64]),
            "sat_tfrecord_frame": (ctypes.c_int64, [_P, _I64, _P]),
            "sat_tfrecord_index": (ctypes.c_int64, [_P, _I64, _I32, _P, _I64])}

_lib: Optional[ctypes.CDLL] = None
# include/sat_abi.h SAT_ABI_VERSION this binding's structs follow
ABI_VERSION = 8


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SatLibraryError(f"{path} not found: run __graft_entry__.build() (make -C csrc)")
    lib = ctypes.CDLL(path)
    # the structs / signatures below are bound with THIS binding's layout: refuse a library
    # built against another (an older build loaded through SAT_LIB_OVERRIDE for an A/B would
    # otherwise read past a struct that has since lost or gained fields)
    got = lib.sat_abi_version() if hasattr(lib, "sat_abi_version") else None
    if got != ABI_VERSION:
        raise SatLibraryError(f"{path}: ABI version {got}, this binding needs {ABI_VERSION} "
                              "(rebuild it: make -C self-attention-tacotron_amd/csrc)")
    # (an A/B build loaded through SAT_LIB_OVERRIDE must therefore carry this ABI version too)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    lib.sat_last_error_string.argtypes = []
    lib.sat_last_error_string.restype = ctypes.c_char_p
    for name, (res, argtypes) in RESTYPES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = res
    _lib = lib
    return lib


HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "sat_abi.h")


def bound_symbols():
    """Entry points this binding declares argtypes for."""
    return set(SIGNATURES) | set(RESTYPES) | {"sat_last_error_string"}


def header_symbols(path: str = HEADER_PATH):
    """Function names declared in include/sat_abi.h (comments stripped)."""
    import re
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return set(re.findall(r"\b(sat_\w+)\s*\(", text))


def exported_symbols(path: str = LIB_PATH):
    """Header symbols the shared library actually exports (dlsym; no device call is made)."""
    lib = ctypes.CDLL(path)
    out = set()
    for name in header_symbols():
        try:
            getattr(lib, name)
            out.add(name)
        except AttributeError:
            pass
    return out


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().sat_last_error_string().decode(errors="replace")
        raise SatLibraryError(f"{what} failed (rc={rc}): {msg}", rc)


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)
