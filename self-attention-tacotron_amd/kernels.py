"""Thin typed wrappers: torch device tensors -> C-ABI calls of libsat_hip.so.

Every function launches on the current torch HIP stream (so a ``torch.cuda.graph`` capture
records it) and never synchronises or allocates outside torch's allocator.
"""

from __future__ import annotations

import ctypes

import torch

from . import _lib

ACT = {None: 0, "none": 0, "relu": 1, "tanh": 2, "sigmoid": 3}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t) -> int:
    return 0 if t is None else t.data_ptr()


def _f32(t, name):
    if t is not None and (t.dtype != torch.float32 or not t.is_cuda):
        raise TypeError(f"{name}: expected a float32 device tensor, got {t.dtype} on {t.device}")


def gemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor = None, *, alpha=1.0, beta=0.0,
         bias=None, act=None, mul=None) -> torch.Tensor:
    """C = act(alpha * A @ B + beta * C + bias).  A [.., M, K], B [.., K, N] (any strides: pass
    ``x.t()`` / ``x.transpose(-1,-2)`` views for transposed operands), optional batch dim 0."""
    _f32(A, "A"); _f32(B, "B")
    batched = A.dim() == 3 or B.dim() == 3
    M, K = A.shape[-2], A.shape[-1]
    K2, N = B.shape[-2], B.shape[-1]
    if K != K2:
        raise ValueError(f"gemm: inner dims differ {A.shape} @ {B.shape}")
    nb = A.shape[0] if A.dim() == 3 else (B.shape[0] if B.dim() == 3 else 1)
    if C is None:
        C = torch.empty((nb, M, N) if batched else (M, N), device=A.device, dtype=torch.float32)
        if beta != 0.0:
            raise ValueError("beta != 0 needs an output tensor")
    _f32(C, "C")
    if C.stride(-1) != 1:
        raise ValueError("gemm: C must have unit column stride")
    d = _lib.SatGemmDesc()
    d.M, d.N, d.K, d.batch = M, N, K, nb
    d.a_mode = 0
    d.A = _p(A)
    d.a_sm, d.a_sk = A.stride(-2), A.stride(-1)
    d.a_sbatch = A.stride(0) if A.dim() == 3 else 0
    d.b_mode = 0
    d.B = _p(B)
    d.b_sk, d.b_sn = B.stride(-2), B.stride(-1)
    d.b_sbatch = B.stride(0) if B.dim() == 3 else 0
    d.C = _p(C)
    d.c_sm = C.stride(-2)
    d.c_sbatch = C.stride(0) if C.dim() == 3 else 0
    d.bias = _p(bias)
    d.bias_sbatch = 0
    d.act = ACT[act]
    d.alpha, d.beta = alpha, beta
    if mul is not None:
        d.mul, d.mul_sm = _p(mul), mul.stride(-2)
        d.mul_sbatch = mul.stride(0) if mul.dim() == 3 else 0
    _lib.check(_lib.load().sat_gemm(ctypes.byref(d), _stream()), "sat_gemm")
    return C


def linear(x: torch.Tensor, W: torch.Tensor, bias=None, act=None, out=None, beta=0.0,
           mul=None):
    """tf.layers.Dense over the last dim of x (any leading shape; x must be row-contiguous);
    ``mul`` (same shape as the output) is multiplied in after the activation (dropout)."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    o2 = None if out is None else out.view(-1, W.shape[1])
    m2 = None if mul is None else mul.reshape(-1, W.shape[1])
    y = gemm(x2, W, o2, bias=bias, act=act, beta=beta, mul=m2)
    return y.view(*lead, W.shape[1])


def conv1d(x: torch.Tensor, W: torch.Tensor, bias=None, out=None, act=None, beta=0.0):
    """Conv1D(SAME, stride 1), x [S, L, Cin] contiguous, W [taps, Cin, Cout] -> [S, L, Cout]."""
    S, L, Cin = x.shape
    taps, Cin2, Cout = W.shape
    assert Cin == Cin2 and x.is_contiguous() and W.is_contiguous()
    if out is None:
        out = torch.empty(S, L, Cout, device=x.device, dtype=torch.float32)
    d = _lib.SatGemmDesc()
    d.M, d.N, d.K, d.batch = S * L, Cout, taps * Cin, 1
    d.a_mode, d.a_L, d.a_C, d.a_shift = 1, L, Cin, (taps - 1) // 2
    d.A, d.a_sm, d.a_sk = _p(x), Cin, 1
    d.b_mode, d.B, d.b_sk, d.b_sn = 0, _p(W), Cout, 1
    d.C, d.c_sm = _p(out), out.stride(1)
    d.bias, d.act, d.alpha, d.beta = _p(bias), ACT[act], 1.0, beta
    _lib.check(_lib.load().sat_gemm(ctypes.byref(d), _stream()), "sat_gemm(conv1d)")
    return out


def conv1d_dx(dy: torch.Tensor, W: torch.Tensor, out=None, beta=0.0):
    """Gradient of conv1d wrt its input: dy [S, L, Cout] -> dx [S, L, Cin]."""
    S, L, Cout = dy.shape
    taps, Cin, _ = W.shape
    if out is None:
        out = torch.empty(S, L, Cin, device=dy.device, dtype=torch.float32)
    d = _lib.SatGemmDesc()
    d.M, d.N, d.K, d.batch = S * L, Cin, taps * Cout, 1
    d.a_mode, d.a_L, d.a_C, d.a_shift = 1, L, Cout, taps - 1 - (taps - 1) // 2
    d.A, d.a_sm, d.a_sk = _p(dy), Cout, 1
    d.b_mode, d.b_taps, d.b_C, d.B = 1, taps, Cout, _p(W)
    d.C, d.c_sm = _p(out), out.stride(1)
    d.alpha, d.beta = 1.0, beta
    _lib.check(_lib.load().sat_gemm(ctypes.byref(d), _stream()), "sat_gemm(conv1d_dx)")
    return out


def conv1d_dw(x: torch.Tensor, dy: torch.Tensor, dW: torch.Tensor, beta=0.0):
    """Gradient of conv1d wrt its kernel: dW [taps, Cin, Cout] = im2col(x)^T @ dy."""
    S, L, Cin = x.shape
    taps, _, Cout = dW.shape
    d = _lib.SatGemmDesc()
    d.M, d.N, d.K, d.batch = taps * Cin, Cout, S * L, 1
    d.a_mode, d.a_L, d.a_C, d.a_shift = 2, L, Cin, (taps - 1) // 2
    d.A, d.a_sm, d.a_sk = _p(x), Cin, 1
    d.b_mode, d.B, d.b_sk, d.b_sn = 0, _p(dy), Cout, 1
    d.C, d.c_sm = _p(dW), Cout
    d.alpha, d.beta = 1.0, beta
    _lib.check(_lib.load().sat_gemm(ctypes.byref(d), _stream()), "sat_gemm(conv1d_dw)")
    return dW


def rng_fill(out: torch.Tensor, seed_dev: torch.Tensor, stream_id: int, keep: float,
             on_value: float):
    _lib.call("sat_rng_fill", _p(out), out.numel(), _p(seed_dev), stream_id, keep, on_value,
              _stream())
    return out


def seq_mask(x: torch.Tensor, lengths: torch.Tensor, out=None):
    B, N, C = x.shape
    if out is None:
        out = torch.empty_like(x)
    _lib.call("sat_seq_mask", _p(x), _p(out), B, N, C, _p(lengths), _stream())
    return out


def _rs(t) -> int:
    """row stride (elements) of a 2-D view"""
    return 0 if t is None else t.stride(0)


def lstm_step_fwd(*, B, U, K, t, xproj, rin, W, c_prev, h_prev, mask_c, mask_h, zc, zh,
                  h_raw, c_out, h_out, gates, lengths=None, bias=None):
    a = _lib.SatLstmFwd()
    a.B, a.U, a.K, a.t = B, U, K, t
    a.xproj, a.xproj_sb = _p(xproj), _rs(xproj)
    a.bias = _p(bias)
    a.rin, a.rin_sb = _p(rin), _rs(rin)
    a.W = _p(W)
    a.c_prev = _p(c_prev)
    a.h_prev, a.h_prev_sb = _p(h_prev), _rs(h_prev)
    a.mask_c, a.mask_h = _p(mask_c), _p(mask_h)
    a.zc, a.zh = zc, zh
    a.lengths = _p(lengths)
    a.h_raw, a.h_raw_sb = _p(h_raw), _rs(h_raw)
    a.c_out = _p(c_out)
    a.h_out, a.h_out_sb = _p(h_out), _rs(h_out)
    a.gates = _p(gates)
    _lib.check(_lib.load().sat_lstm_step_fwd(ctypes.byref(a), _stream()), "sat_lstm_step_fwd")


def lstm_step_bwd(*, B, U, K, hoff, t, W, dgates_next, gates, c_prev, dy, dh_carry, dc_carry,
                  mask_c, mask_h, zc, zh, dgates, dh_carry_out, dc_carry_out, lengths=None,
                  dq0=None, wq0=None, dq1=None, wq1=None):
    a = _lib.SatLstmBwd()
    a.B, a.U, a.K, a.hoff, a.t = B, U, K, hoff, t
    a.W, a.dgates_next, a.gates, a.c_prev = _p(W), _p(dgates_next), _p(gates), _p(c_prev)
    a.dy, a.dy_sb = _p(dy), _rs(dy)
    a.dq0, a.wq0, a.dq0_n = _p(dq0), _p(wq0), 0 if dq0 is None else dq0.shape[-1]
    a.dq1, a.wq1, a.dq1_n = _p(dq1), _p(wq1), 0 if dq1 is None else dq1.shape[-1]
    a.dh_carry, a.dc_carry = _p(dh_carry), _p(dc_carry)
    a.mask_c, a.mask_h = _p(mask_c), _p(mask_h)
    a.zc, a.zh = zc, zh
    a.lengths = _p(lengths)
    a.dgates, a.dh_carry_out, a.dc_carry_out = _p(dgates), _p(dh_carry_out), _p(dc_carry_out)
    _lib.check(_lib.load().sat_lstm_step_bwd(ctypes.byref(a), _stream()), "sat_lstm_step_bwd")


def attn_query(x, W1, W2, q):
    B, K = x.shape
    _lib.call("sat_attn_query", B, K, W1.shape[1], 0 if W2 is None else W2.shape[1], _p(x),
              _rs(x), _p(W1), _p(W2), _p(q), _rs(q), _stream())


def part_stride(M1, M2) -> int:
    return _lib.load().sat_attn_part_stride(M1, M2)


def attn_step_fwd(**kw):
    a = _lib.SatAttnStep()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_attn_step_fwd(ctypes.byref(a), _stream()), "sat_attn_step_fwd")
