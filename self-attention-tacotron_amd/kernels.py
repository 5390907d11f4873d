"""Thin typed wrappers: torch device tensors -> C-ABI calls of libsat_hip.so.

Every function launches on the current torch HIP stream (so a ``torch.cuda.graph`` capture
records it) and never synchronises or allocates outside torch's allocator.
"""

from __future__ import annotations

import ctypes
import os

import torch

from . import _lib

ACT = {None: 0, "none": 0, "relu": 1, "tanh": 2, "sigmoid": 3, "softsign": 4}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t) -> int:
    return 0 if t is None else t.data_ptr()


_GEMM_WS = {}
GEMM_WS_BYTES = 32 << 20


def _gemm_ws(device):
    """Split-K scratch, one per (device, stream): GEMMs on concurrent pipeline lanes never share
    it.  Allocated on first use on that stream (the eager warm-up, before graph capture)."""
    key = (device.type, device.index, torch.cuda.current_stream(device).cuda_stream)
    buf = _GEMM_WS.get(key)
    if buf is None:
        buf = torch.empty(GEMM_WS_BYTES, dtype=torch.uint8, device=device)
        _GEMM_WS[key] = buf
    return buf


_SCRATCH = {}


def _stream_scratch(device, tag: str, nbytes: int) -> int:
    """Small fixed-size device scratch per (device, stream, tag), allocated on first use."""
    key = (device.type, device.index, torch.cuda.current_stream(device).cuda_stream, tag)
    buf = _SCRATCH.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _SCRATCH[key] = buf
    return buf.data_ptr()


_AUX = {}


def aux_stream(device, which: int = 0) -> torch.cuda.Stream:
    """The step's second stream (independent branches beside the encoder, forward and backward),
    one per device, made on first use -- the eager warm-up before any graph capture; the GEMM
    split-K and column-reduction scratch are keyed per stream already.  ``which=1``: a third
    stream (the encoder backward's weight-gradient branches, SAT_AUX2=1)."""
    key = (device.index, which)
    s = _AUX.get(key)
    if s is None:
        s = _AUX[key] = torch.cuda.Stream(device=device)
    return s


# Optional launch log for tools/gemm_census.py: list of (tag, SatGemmDesc copy, call site) when
# not None.
GEMM_LOG = None


def _call_site() -> str:
    import traceback
    for fr in reversed(traceback.extract_stack()[:-2]):
        if not fr.filename.endswith("kernels.py"):
            return f"{os.path.basename(fr.filename)}:{fr.lineno}:{fr.name}"
    return "?"


def _launch_gemm(d, tag):
    if GEMM_LOG is not None:
        GEMM_LOG.append((tag, type(d).from_buffer_copy(d), _call_site()))
    _lib.check(_lib.load().sat_gemm(ctypes.byref(d), _stream()), tag)


def _with_ws(d, device):
    buf = _gemm_ws(device)
    d.ws, d.ws_bytes = buf.data_ptr(), buf.numel()


def _f32(t, name):
    if t is not None and (t.dtype != torch.float32 or not t.is_cuda):
        raise TypeError(f"{name}: expected a float32 device tensor, got {t.dtype} on {t.device}")


def _bstrides(t, nd):
    """batch strides (s1, s2) of a tensor with nd leading batch dims (0 = broadcast)."""
    if t is None:
        return 0, 0
    lead = t.dim() - 2
    if lead == 2:
        return t.stride(0), t.stride(1)
    if lead == 1:
        return (t.stride(0), 0) if nd >= 1 else (0, 0)
    return 0, 0


def gemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor = None, *, alpha=1.0, beta=0.0,
         bias=None, act=None, mul=None, add=None, colsum=None, A2=None, C2=None,
         B2=None, tri=0) -> torch.Tensor:
    """C = act(alpha * A @ B + beta * C + bias) * mul + add.

    ``A2`` [M, K2] (2-D, row-contiguous like A): A is the two column blocks [A | A2] of one
    reduction over B [K1 + K2, N] (SatGemmDesc.A2: two inputs of a layer in different buffers).
    ``C2`` [M, N - N1] (2-D, unit column stride): the product's columns split between C [M, N1]
    and C2 (SatGemmDesc.C2: two outputs of one A over the column blocks of one B).
    ``B2`` [K2, N] (B's layout): B is the two row blocks [B ; B2] of one reduction; with ``A2``
    the launch computes A B + A2 B2 (SatGemmDesc.B2).

    ``tri`` (SatGemmDesc.tri, a hint for a causal attention's per-batch square products): 1 only
    the lower triangle of C is needed (tiles above the diagonal left unwritten); 2 / 3 A is
    lower / upper triangular (its zero K-tiles are not loaded: same bits).

    ``colsum`` [N] (2-D, plain products only): also colsum = alpha * sum over rows of B + beta *
    colsum in the same launch (a dense layer's bias gradient next to its weight gradient); with
    one batch dim, [batch, N]: one row per batch.

    A [.., M, K], B [.., K, N] with up to two leading batch dims (any strides: pass ``x.t()`` /
    ``x.transpose(-1, -2)`` views for transposed operands); C gets the broadcast batch shape.
    """
    _f32(A, "A"); _f32(B, "B")
    M, K = A.shape[-2], A.shape[-1]
    k1 = K
    if A2 is not None:
        _f32(A2, "A2")
        if (A2.shape[:-1] != A.shape[:-1] or A2.stride(-1) != 1 or
                A2.stride()[:-2] != A.stride()[:-2]):
            raise ValueError("gemm: A2 must be [.., M, K2] with A's batch shape and strides and "
                             "unit column stride")
        K = k1 + A2.shape[-1]
    K2, N = B.shape[-2], B.shape[-1]
    if B2 is not None:
        _f32(B2, "B2")
        if (B2.shape[:-2] != B.shape[:-2] or B2.shape[-1] != N or
                B2.stride()[:-2] != B.stride()[:-2] or
                (B.stride(-1) == 1) != (B2.stride(-1) == 1) or (A2 is not None and K2 != k1)):
            raise ValueError("gemm: B2 must be [.., K2, N] in B's layout and batch strides, "
                             "beside B [.., k1, N]")
        k1 = K2
        K2 += B2.shape[-2]
    if K != K2:
        raise ValueError(f"gemm: inner dims differ {tuple(A.shape)} @ {tuple(B.shape)}")
    lead = A.shape[:-2] if A.dim() >= B.dim() else B.shape[:-2]
    if len(lead) > 2:
        raise ValueError("gemm: at most two batch dims")
    if C is None:
        if beta != 0.0:
            raise ValueError("beta != 0 needs an output tensor")
        C = torch.empty((*lead, M, N), device=A.device, dtype=torch.float32)
    _f32(C, "C")
    if C.stride(-1) != 1:
        raise ValueError("gemm: C must have unit column stride")
    nd = len(lead)
    nb = lead[0] if nd >= 1 else 1
    nb2 = lead[1] if nd == 2 else 1
    d = _lib.SatGemmDesc()
    d.M, d.N, d.K, d.batch, d.batch2 = M, N, K, nb, nb2
    d.a_mode, d.A = 0, _p(A)
    d.a_sm, d.a_sk = A.stride(-2), A.stride(-1)
    d.a_sbatch, d.a_sbatch2 = _bstrides(A, nd)
    d.b_mode, d.B = 0, _p(B)
    d.b_sk, d.b_sn = B.stride(-2), B.stride(-1)
    d.b_sbatch, d.b_sbatch2 = _bstrides(B, nd)
    d.C, d.c_sm = _p(C), C.stride(-2)
    d.c_sbatch, d.c_sbatch2 = _bstrides(C, nd)
    d.bias, d.bias_sbatch = _p(bias), (bias.stride(0) if bias is not None and bias.dim() == 2
                                       else 0)
    d.act = ACT[act]
    d.alpha, d.beta = alpha, beta
    if mul is not None:
        d.mul, d.mul_sm = _p(mul), mul.stride(-2)
        d.mul_sbatch, d.mul_sbatch2 = _bstrides(mul, nd)
    if add is not None:
        d.add = _p(add)
        d.add_sm = add.stride(-2) if add.dim() >= 2 else 0
        d.add_sbatch = add.stride(0) if add.dim() == 3 else 0
    if colsum is not None:
        _f32(colsum, "colsum")
        if nd == 1 and colsum.dim() == 2:       # one [N] row per batch (bias_sbatch apart)
            if tuple(colsum.shape) != (nb, N) or colsum.stride(1) != 1:
                raise ValueError("gemm: a batched colsum must be [batch, N] with unit stride")
            d.bias_sbatch = colsum.stride(0)
        elif colsum.numel() != N or not colsum.is_contiguous():
            raise ValueError("gemm: colsum must be a contiguous [N] tensor")
        elif nb > 1 and d.b_sbatch != 0:
            # one [N] row with a batched B would keep batch 0's column sums only
            raise ValueError("gemm: a batched product with a batch-strided B needs a "
                             "[batch, N] colsum")
        d.colsum_out = _p(colsum)
    if A2 is not None:
        d.A2, d.a2_sm, d.k1 = _p(A2), A2.stride(-2), k1
    if B2 is not None:
        d.B2, d.k1 = _p(B2), k1
        d.b2_s = B2.stride(-2) if B2.stride(-1) == 1 else B2.stride(-1)
    if C2 is not None:
        _f32(C2, "C2")
        if nd != 0 or C.dim() != 2 or C2.dim() != 2 or C2.stride(1) != 1 or C2.shape[0] != M or \
                C.shape[1] + C2.shape[1] != N:
            raise ValueError("gemm: C2 must be [M, N - N1] beside a 2-D C [M, N1]")
        d.C2, d.c2_sm, d.n1 = _p(C2), C2.stride(0), C.shape[1]
    d.tri = int(tri)
    _with_ws(d, C.device)
    _launch_gemm(d, "sat_gemm")
    return C


def gemm_wgrad_batch(Xs, dY: torch.Tensor, dWs, colsum=None, beta=1.0):
    """dW_b = X_b^T dY + beta dW_b for every b as ONE batched launch (split-K over the batches'
    slabs): the weight gradients of layers that share the output gradient dY [K, N] (the blocks
    of one LSTM kernel).  Xs: 2-D [K, M] views of one shape and strides, equally spaced in
    memory (any buffers); dWs: [M, N] row-contiguous, equally spaced.  ``colsum`` [N]: also
    colsum = sum over rows of dY + beta colsum, once (SatGemmDesc.colsum_out, bias_sbatch 0)."""
    nb = len(Xs)
    X0, W0 = Xs[0], dWs[0]
    for t in list(Xs) + [dY] + list(dWs):
        _f32(t, "gemm_wgrad_batch operand")
    K_, M = X0.shape
    N = dY.shape[1]
    sx = (Xs[1].data_ptr() - X0.data_ptr()) // 4 if nb > 1 else 0
    sw = (dWs[1].data_ptr() - W0.data_ptr()) // 4 if nb > 1 else 0
    for b in range(nb):
        X, W = Xs[b], dWs[b]
        if (tuple(X.shape) != (K_, M) or X.stride() != X0.stride() or
                X.data_ptr() - X0.data_ptr() != 4 * b * sx or tuple(W.shape) != (M, N) or
                W.stride() != W0.stride() or W.stride(1) != 1 or
                W.data_ptr() - W0.data_ptr() != 4 * b * sw or dY.shape[0] != K_):
            raise ValueError("gemm_wgrad_batch: operands must share shape / strides and be "
                             "equally spaced")
    d = _lib.SatGemmDesc()
    d.M, d.N, d.K, d.batch, d.batch2 = M, N, K_, nb, 1
    d.A, d.a_sm, d.a_sk, d.a_sbatch = _p(X0), X0.stride(1), X0.stride(0), sx
    d.B, d.b_sk, d.b_sn, d.b_sbatch = _p(dY), dY.stride(0), dY.stride(1), 0
    d.C, d.c_sm, d.c_sbatch = _p(W0), W0.stride(0), sw
    d.alpha, d.beta = 1.0, beta
    d.batch2 = 1
    if colsum is not None:
        _f32(colsum, "colsum")
        if colsum.numel() != N or not colsum.is_contiguous():
            raise ValueError("gemm_wgrad_batch: colsum must be a contiguous [N] tensor")
        d.colsum_out = _p(colsum)
    _with_ws(d, dY.device)
    _launch_gemm(d, "sat_gemm")


def rowdot(A: torch.Tensor, Bt: torch.Tensor, C: torch.Tensor, alpha=1.0, beta=0.0):
    """C = alpha * A @ Bt^T + beta * C  (A [M, K], Bt [N, K] row-contiguous)."""
    M, Kd = A.shape
    N = Bt.shape[0]
    _lib.call("sat_gemm_rowdot", M, N, Kd, _p(A), A.stride(0), _p(Bt), Bt.stride(0), _p(C),
              C.stride(0), alpha, beta, _stream())
    return C


def linear(x: torch.Tensor, W: torch.Tensor, bias=None, act=None, out=None, beta=0.0,
           mul=None, add=None):
    """tf.layers.Dense over the last dim of x (any leading shape; x must be row-contiguous);
    ``mul`` (same shape as the output) is multiplied in after the activation (dropout), ``add``
    added last (residual)."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    o2 = None if out is None else out.view(-1, W.shape[1])
    m2 = None if mul is None else mul.reshape(-1, W.shape[1])
    a2 = None if add is None else add.reshape(-1, W.shape[1])
    y = gemm(x2, W, o2, bias=bias, act=act, beta=beta, mul=m2, add=a2)
    return y.view(*lead, W.shape[1])


def conv1d(x: torch.Tensor, W: torch.Tensor, bias=None, out=None, act=None, beta=0.0):
    """Conv1D(SAME, stride 1), x [S, L, Cin] contiguous, W [taps, Cin, Cout] -> [S, L, Cout]."""
    S, L, Cin = x.shape
    taps, Cin2, Cout = W.shape
    assert Cin == Cin2 and x.stride(2) == 1 and x.stride(0) == L * x.stride(1)
    assert W.is_contiguous()
    if out is None:
        out = torch.empty(S, L, Cout, device=x.device, dtype=torch.float32)
    d = _lib.SatGemmDesc()
    d.M, d.N, d.K, d.batch = S * L, Cout, taps * Cin, 1
    d.a_mode, d.a_L, d.a_C, d.a_shift = 1, L, Cin, (taps - 1) // 2
    d.A, d.a_sm, d.a_sk = _p(x), x.stride(1), 1
    d.b_mode, d.B, d.b_sk, d.b_sn = 0, _p(W), Cout, 1
    d.C, d.c_sm = _p(out), out.stride(1)
    d.bias, d.act, d.alpha, d.beta = _p(bias), ACT[act], 1.0, beta
    _with_ws(d, x.device)
    _launch_gemm(d, "sat_gemm(conv1d)")
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
    d.A, d.a_sm, d.a_sk = _p(dy), dy.stride(1), 1
    d.b_mode, d.b_taps, d.b_C, d.B = 1, taps, Cout, _p(W)
    d.C, d.c_sm = _p(out), out.stride(1)
    d.alpha, d.beta = 1.0, beta
    _with_ws(d, dy.device)
    _launch_gemm(d, "sat_gemm(conv1d_dx)")
    return out


def conv1d_dw(x: torch.Tensor, dy: torch.Tensor, dW: torch.Tensor, beta=0.0):
    """Gradient of conv1d wrt its kernel: dW [taps, Cin, Cout] = im2col(x)^T @ dy."""
    S, L, Cin = x.shape
    taps, _, Cout = dW.shape
    d = _lib.SatGemmDesc()
    d.M, d.N, d.K, d.batch = taps * Cin, Cout, S * L, 1
    d.a_mode, d.a_L, d.a_C, d.a_shift = 2, L, Cin, (taps - 1) // 2
    d.A, d.a_sm, d.a_sk = _p(x), x.stride(1), 1
    d.b_mode, d.B, d.b_sk, d.b_sn = 0, _p(dy), dy.stride(1), 1
    d.C, d.c_sm = _p(dW), Cout
    d.alpha, d.beta = 1.0, beta
    _with_ws(d, dW.device)
    _launch_gemm(d, "sat_gemm(conv1d_dw)")
    return dW



def _bank_desc(x, W_bank, max_k, Co, y):
    S, L, C = x.shape
    assert x.stride(2) == 1 and x.stride(0) == L * x.stride(1)
    assert y.stride(-1) == 1 and y.stride(0) == L * y.stride(1) and y.shape[-1] == max_k * Co
    assert W_bank.is_contiguous() and W_bank.numel() == Co * C * max_k * (max_k + 1) // 2
    d = _lib.SatConvBank()
    d.S, d.L, d.C, d.max_k, d.Co = S, L, C, max_k, Co
    d.x, d.x_sm, d.W = _p(x), x.stride(1), _p(W_bank)
    d.y, d.y_sm = _p(y), y.stride(1)
    return d


def conv_bank(x: torch.Tensor, W_bank: torch.Tensor, bias, y: torch.Tensor, max_k: int, Co: int):
    """CBHG conv bank (modules/module.py:77-80): y[:, :, (k-1)Co:kCo] = Conv1D_k(x) + b_k for
    k = 1..max_k in ONE launch.  W_bank = K1..Kmax kernels back to back ([k][C][Co] each)."""
    d = _bank_desc(x, W_bank, max_k, Co, y)
    d.bias = _p(bias)
    _lib.check(_lib.load().sat_cbhg_convbank_fwd(ctypes.byref(d), _stream()),
               "sat_cbhg_convbank_fwd")
    return y


def conv_bank_bwd(x, W_bank, dy, max_k: int, Co: int, dx=None, dW=None, beta_dx=0.0,
                  beta_dw=1.0):
    """Both gradients of conv_bank: dx (= beta_dx dx + sum_k conv_dx_k) and dW (accumulated with
    beta_dw), each ONE product over the whole bank (split-K scratch from the stream pool)."""
    d = _bank_desc(x, W_bank, max_k, Co, dy)
    if dx is not None:
        assert dx.stride(-1) == 1 and dx.shape == x.shape
        d.dx, d.dx_sm, d.beta_dx = _p(dx), dx.stride(1), beta_dx
    if dW is not None:
        assert dW.is_contiguous() and dW.numel() == W_bank.numel()
        d.dW, d.beta_dw = _p(dW), beta_dw
    _with_ws(d, x.device)
    _lib.check(_lib.load().sat_cbhg_convbank_bwd(ctypes.byref(d), _stream()),
               "sat_cbhg_convbank_bwd")

def decode_attention_step(qkv: torch.Tensor, t: int, H: int, D: int, scale: float,
                          P: torch.Tensor, O: torch.Tensor):
    """sat_decode_attention_step: qkv [B, Tm, 3D] cache (row t written), P [B, H, Tm, Tm]
    probability rows (row t written), O [B, D] the heads' outputs."""
    B, Tm = qkv.shape[0], qkv.shape[1]
    _lib.call("sat_decode_attention_step", _p(qkv), qkv.stride(0), qkv.stride(1), B, H, D, t,
              scale, _p(P), Tm if P is not None else 0, _p(O), O.stride(0), _stream())


def decode_persistent_scratch_bytes() -> int:
    return int(_lib.load().sat_decode_persistent_scratch_bytes())


def decode_persistent(**kw):
    """sat_decode_persistent: the whole free-running decode as one launch (tensor arguments by
    the SatDecodePersistent field names, scalars as ints / floats)."""
    d = _lib.SatDecodePersistent()
    for k, v in kw.items():
        setattr(d, k, _p(v) if isinstance(v, torch.Tensor) or v is None else v)
    _lib.check(_lib.load().sat_decode_persistent(ctypes.byref(d), _stream()),
               "sat_decode_persistent")


def stop_check(stop: torch.Tensor, t: int, min_iters: int, state: torch.Tensor):
    """state[0] := t if (no earlier finish) and t > min_iters and all sigmoid(stop) > 0.5."""
    _lib.call("sat_stop_check", _p(stop), stop.stride(0), stop.shape[0], t, min_iters,
              _p(state), _stream())


def empty_group(*shapes, device):
    """zeros_group's carving without the fill: (buffer, pieces); the caller zeroes ``buffer``
    (e.g. on a side stream, off the critical path)."""
    sizes = [int(torch.Size(sh).numel()) for sh in shapes]
    pads = [(n + 63) // 64 * 64 for n in sizes]
    buf = torch.empty(sum(pads), device=device, dtype=torch.float32)
    out, off = [], 0
    for sh, n, pn in zip(shapes, sizes, pads):
        out.append(buf[off:off + n].view(sh))
        off += pn
    return buf, out


def fill_(t: torch.Tensor, value: float = 0.0) -> torch.Tensor:
    """t[...] = value (float32 or int32 device tensor, contiguous) with sat_fill32 -- the
    captured step's zero-initialised buffers and error words without a framework fill."""
    if not t.is_contiguous() or t.element_size() != 4 or not t.is_cuda:
        raise ValueError("fill_: contiguous 4-byte device tensor expected")
    if t.dtype == torch.float32:
        bits = ctypes.c_uint32.from_buffer(ctypes.c_float(value)).value
    elif t.dtype == torch.int32:
        bits = int(value) & 0xFFFFFFFF
    else:
        raise ValueError(f"fill_: unsupported dtype {t.dtype}")
    _lib.call("sat_fill32", _p(t), t.numel(), bits, _stream())
    return t


def zeros(*shape, device, dtype=torch.float32) -> torch.Tensor:
    """torch.zeros without the framework fill kernel (sat_fill32)."""
    return fill_(torch.empty(*shape, device=device, dtype=dtype))


def copy3d_(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """dst[...] = src[...] for same-shape tensors of up to 3 dims with unit innermost strides
    (a transposed view made contiguous, a strided slice into a step buffer) -- sat_copy3d."""
    if dst.shape != src.shape or dst.dim() > 3 or dst.dtype != torch.float32 or \
            src.dtype != torch.float32:
        raise ValueError("copy3d_: same-shape float32 tensors of <= 3 dims expected")
    shp = [1] * (3 - dst.dim()) + list(dst.shape)
    ss = [0] * (3 - src.dim()) + list(src.stride())
    ds = [0] * (3 - dst.dim()) + list(dst.stride())
    if shp[2] > 1 and (ss[2] != 1 or ds[2] != 1):
        raise ValueError("copy3d_: unit innermost strides expected")
    _lib.call("sat_copy3d", _p(src), ss[0], ss[1], _p(dst), ds[0], ds[1], shp[0], shp[1], shp[2],
              _stream())
    return dst


def add(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """x + y (same-shape contiguous float32) as one sat_add launch."""
    if x.shape != y.shape or not (x.is_contiguous() and y.is_contiguous()):
        raise ValueError("add: same-shape contiguous tensors expected")
    z = torch.empty_like(x)
    _lib.call("sat_add", _p(x), _p(y), _p(z), x.numel(), _stream())
    return z


_ONES = {}


def ones(*shape, device) -> torch.Tensor:
    """A cached read-only float32 tensor of ones (made once per device, before any capture)."""
    n = int(torch.Size(shape).numel())
    dev = torch.device(device)
    buf = _ONES.get(dev)
    if buf is None or buf.numel() < n:
        buf = _ONES[dev] = torch.ones(max(n, 4096), device=dev)
    return buf[:n].view(*shape)


def contiguous(x: torch.Tensor) -> torch.Tensor:
    """x made contiguous with sat_copy3d (x itself when it already is)."""
    if x.is_contiguous():
        return x
    return copy3d_(torch.empty(x.shape, device=x.device, dtype=x.dtype), x)


def zeros_group(*shapes, device):
    """Several zero-initialised float32 tensors carved from ONE zeroed buffer (one fill launch
    instead of one per tensor in the captured step); every piece starts on a 256-byte boundary
    (the kernels' 16-byte operand alignment)."""
    sizes = [int(torch.Size(sh).numel()) for sh in shapes]
    pads = [(n + 63) // 64 * 64 for n in sizes]
    buf = zeros(sum(pads), device=device)
    out, off = [], 0
    for sh, n, pn in zip(shapes, sizes, pads):
        out.append(buf[off:off + n].view(sh))
        off += pn
    return out


def rng_fill(out: torch.Tensor, seed_dev: torch.Tensor, stream_id: int, keep: float,
             on_value: float):
    _lib.call("sat_rng_fill", _p(out), out.numel(), _p(seed_dev), stream_id, keep, on_value,
              _stream())
    return out


def rng_segments(specs):
    """ctypes array of SatRngSegment from (offset, n, stream_id, keep, on_value) tuples."""
    arr = (_lib.SatRngSegment * len(specs))()
    for i, (off, n, sid, keep, on) in enumerate(specs):
        arr[i].offset, arr[i].n, arr[i].stream_id = off, n, sid
        arr[i].keep, arr[i].on_value = keep, on
    return arr


def rng_fill_segments(base: torch.Tensor, segs, seed_dev: torch.Tensor):
    """Every segment of ``base`` (a flat float32 arena) in ONE launch, each drawing exactly what
    rng_fill on its own view with the same stream id would draw."""
    _lib.call("sat_rng_fill_segments", _p(base), segs, len(segs), _p(seed_dev), _stream())
    return base


def seq_mask(x: torch.Tensor, lengths: torch.Tensor, out=None):
    B, N, C = x.shape
    if out is None:
        out = torch.empty_like(x)
    _lib.call("sat_seq_mask", _p(x), _p(out), B, N, C, _p(lengths), _stream())
    return out


def _rs(t) -> int:
    """row stride (elements) of a 2-D view"""
    return 0 if t is None else t.stride(0)


def lstm_fwd_desc(*, B, U, K, t, xproj, rin, W, c_prev, h_prev, mask_c, mask_h, zc, zh,
                  h_raw, c_out, h_out, gates, lengths=None, bias=None, rin1=None, rin2=None,
                  a=None):
    """Fill a SatLstmFwd (``a``, or a new one) for one recurrent step.  ``rin1`` / ``rin2``:
    further input segments (row = [rin | rin1 | rin2] against W's K rows)."""
    a = _lib.SatLstmFwd() if a is None else a
    a.rin1, a.rin1_sb, a.K1 = _p(rin1), _rs(rin1), 0 if rin1 is None else rin1.shape[-1]
    a.rin2, a.rin2_sb, a.K2 = _p(rin2), _rs(rin2), 0 if rin2 is None else rin2.shape[-1]
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
    return a


def lstm_step_fwd(**kw):
    a = lstm_fwd_desc(**kw)
    _lib.check(_lib.load().sat_lstm_step_fwd(ctypes.byref(a), _stream()), "sat_lstm_step_fwd")


def lstm_steps_fwd(steps):
    """Several independent LSTM steps (list of lstm_step_fwd kwargs) in ONE launch."""
    arr = (_lib.SatLstmFwd * len(steps))()
    for i, kw in enumerate(steps):
        lstm_fwd_desc(a=arr[i], **kw)
    _lib.check(_lib.load().sat_lstm_steps_fwd(arr, len(steps), _stream()), "sat_lstm_steps_fwd")


def lstm_bwd_desc(*, B, U, K, hoff, t, W, dgates_next, gates, c_prev, dy, dh_carry, dc_carry,
                  mask_c, mask_h, zc, zh, dgates, dh_carry_out, dc_carry_out, lengths=None,
                  dq0=None, wq0=None, dq1=None, wq1=None, dq_parts=1, dq_pstride=0,
                  dq_bstride=0, rec=None, a=None):
    a = _lib.SatLstmBwd() if a is None else a
    a.B, a.U, a.K, a.hoff, a.t = B, U, K, hoff, t
    a.W, a.dgates_next, a.gates, a.c_prev = _p(W), _p(dgates_next), _p(gates), _p(c_prev)
    a.dy, a.dy_sb = _p(dy), _rs(dy)
    a.dq0, a.wq0, a.dq0_n = _p(dq0), _p(wq0), 0 if dq0 is None else dq0.shape[-1]
    a.dq1, a.wq1, a.dq1_n = _p(dq1), _p(wq1), 0 if dq1 is None else dq1.shape[-1]
    a.dq_parts, a.dq_pstride, a.dq_bstride = dq_parts, dq_pstride, dq_bstride
    a.dh_carry, a.dc_carry = _p(dh_carry), _p(dc_carry)
    a.mask_c, a.mask_h = _p(mask_c), _p(mask_h)
    a.zc, a.zh = zc, zh
    a.lengths = _p(lengths)
    a.dgates, a.dh_carry_out, a.dc_carry_out = _p(dgates), _p(dh_carry_out), _p(dc_carry_out)
    a.rec, a.rec_sb = _p(rec), _rs(rec)
    return a


def lstm_step_bwd(**kw):
    a = lstm_bwd_desc(**kw)
    _lib.check(_lib.load().sat_lstm_step_bwd(ctypes.byref(a), _stream()), "sat_lstm_step_bwd")


def lstm_steps_bwd(steps):
    """Several independent reverse LSTM steps (list of lstm_step_bwd kwargs) in ONE launch."""
    arr = (_lib.SatLstmBwd * len(steps))()
    for i, kw in enumerate(steps):
        lstm_bwd_desc(a=arr[i], **kw)
    _lib.check(_lib.load().sat_lstm_steps_bwd(arr, len(steps), _stream()), "sat_lstm_steps_bwd")


def attn_query(x, W1, W2, q):
    B, K = x.shape
    _lib.call("sat_attn_query", B, K, W1.shape[1], 0 if W2 is None else W2.shape[1], _p(x),
              _rs(x), _p(W1), _p(W2), _p(q), _rs(q), _stream())


def part_stride(M1, M2) -> int:
    return _lib.load().sat_attn_part_stride(M1, M2)


def attn_param_grad_rows(B: int, N: int) -> int:
    return int(_lib.load().sat_attn_param_grad_rows(B, N))


def attn_param_grads(**kw):
    a = _lib.SatAttnParamGrad()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_attn_param_grads(ctypes.byref(a), _stream()),
               "sat_attn_param_grads")


class DecoderAttentionScratch:
    """Device scratch of sat_decoder_attention_fwd for one (B, N): raw energies, tile partials,
    group counters and the error word (allocated before graph capture)."""

    def __init__(self, B: int, N: int, device, errs: torch.Tensor = None):
        """``errs``: optional int32 device words (>= 8) the four persistent kernels' error pairs
        are carved from (the engine's health arena, read by the guarded Adam step)."""
        if errs is None:
            errs = torch.zeros(8, dtype=torch.int32, device=device)
        self.B, self.N = B, N
        e, pt, qp = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        words = int(_lib.load().sat_decoder_attention_scratch(B, N, ctypes.byref(e),
                                                              ctypes.byref(pt), ctypes.byref(qp)))
        self.E = torch.empty(e.value, device=device)
        self.PART = torch.empty(pt.value, device=device)
        self.QP = torch.empty(qp.value, device=device)
        self.ctr = torch.zeros(words, dtype=torch.int32, device=device)
        self.err = errs[0:2]
        self.bwd = DecoderAttentionBwdScratch(B, N, device, errs[6:8])   # the persistent BPTT's own

        # the persistent decoder LSTM stack's own counters / error words (fwd, bwd)
        self.lstm_xch = torch.zeros(int(_lib.load().sat_decoder_lstms_scratch(B)), device=device)
        self.lstm_ctr = torch.zeros(int(_lib.load().sat_decoder_lstms_bwd_scratch(B)),
                                    dtype=torch.int32, device=device)
        self.lstm_err = errs[2:6].view(2, 2)                                  # fwd, bwd

    def check(self):
        """Host check of the in-kernel barrier timeout flags (synchronises)."""
        if int(self.err[0].item()) != 0:
            raise _lib.SatLibraryError("sat_decoder_attention_fwd: an in-kernel hand-off timed out "
                                       "(workgroups not co-resident?)")
        for i, nm in enumerate(("sat_decoder_lstms_fwd", "sat_decoder_lstms_bwd")):
            if int(self.lstm_err[i, 0].item()) != 0:
                raise _lib.SatLibraryError(f"{nm}: a group barrier timed out "
                                           "(workgroups not co-resident?)")
        self.bwd.check()


def decoder_attention_fwd(**kw):
    a = _lib.SatDecAttnFwd()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_decoder_attention_fwd(ctypes.byref(a), _stream()),
               "sat_decoder_attention_fwd")


class DecoderAttentionBwdScratch:
    """Device scratch of sat_decoder_attention_bwd for one (B, N): row-dot partials, the
    alignment-recursion gradient ping-pong, group counters and the error word."""

    def __init__(self, B: int, N: int, device, err: torch.Tensor = None):
        rdp, ya = ctypes.c_int64(), ctypes.c_int64()
        words = int(_lib.load().sat_decoder_attention_bwd_scratch(B, N, ctypes.byref(rdp),
                                                                  ctypes.byref(ya)))
        self.RDP = torch.empty(rdp.value, device=device)
        self.YA = torch.empty(ya.value, device=device)
        self.ctr = torch.zeros(words, dtype=torch.int32, device=device)
        self.err = torch.zeros(2, dtype=torch.int32, device=device) if err is None else err

    def check(self):
        if int(self.err[0].item()) != 0:
            raise _lib.SatLibraryError("sat_decoder_attention_bwd: an in-kernel hand-off timed out "
                                       "(workgroups not co-resident?)")


def decoder_attention_bwd(**kw):
    a = _lib.SatDecAttnBwd()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_decoder_attention_bwd(ctypes.byref(a), _stream()),
               "sat_decoder_attention_bwd")


def encoder_lstm_fwd(**kw):
    """sat_encoder_lstm_fwd: all steps of both encoder BiLSTM directions in one launch."""
    a = _lib.SatEncLstmFwd()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_encoder_lstm_fwd(ctypes.byref(a), _stream()),
               "sat_encoder_lstm_fwd")


def encoder_lstm_bwd(**kw):
    """sat_encoder_lstm_bwd: the BPTT of both encoder BiLSTM directions in one launch."""
    a = _lib.SatEncLstmBwd()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_encoder_lstm_bwd(ctypes.byref(a), _stream()),
               "sat_encoder_lstm_bwd")


def decoder_lstms_fwd(**kw):
    a = _lib.SatDecLstmFwd()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_decoder_lstms_fwd(ctypes.byref(a), _stream()),
               "sat_decoder_lstms_fwd")


def decoder_lstms_bwd(**kw):
    a = _lib.SatDecLstmBwd()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_decoder_lstms_bwd(ctypes.byref(a), _stream()),
               "sat_decoder_lstms_bwd")


def attn_step_bwd(**kw):
    a = _lib.SatAttnStepBwd()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_attn_step_bwd(ctypes.byref(a), _stream()), "sat_attn_step_bwd")


def pg_stride(D1, D2, F, KW) -> int:
    return _lib.load().sat_attn_pg_stride(D1, D2, F, KW)


def attn_step_fwd(**kw):
    a = _lib.SatAttnStep()
    for k, v in kw.items():
        setattr(a, k, _p(v) if isinstance(v, torch.Tensor) else v)
    _lib.check(_lib.load().sat_attn_step_fwd(ctypes.byref(a), _stream()), "sat_attn_step_fwd")


# ---------------------------------------------------------------- elementwise / reductions

class Workspace:
    """Grow-only fp64 scratch for column reductions, one buffer per stream (pipeline lanes
    reduce concurrently)."""

    def __init__(self, device):
        self.device = device
        self.bufs = {}

    def get(self, M, C) -> int:
        need = int(_lib.load().sat_workspace_colreduce(M, C))
        key = torch.cuda.current_stream(self.device).cuda_stream
        buf = self.bufs.get(key)
        if buf is None or buf.numel() < need:
            old = 0 if buf is None else buf.numel()
            buf = torch.empty(max(need, 2 * old, 1 << 20), dtype=torch.uint8, device=self.device)
            self.bufs[key] = buf
        return buf.data_ptr()


def embedding_fwd(table, ids, out, offset=0, err=None):
    R = ids.numel()
    _lib.call("sat_embedding_fwd", _p(table), _p(ids), _p(out), R, table.shape[1],
              table.shape[0], offset, _p(err), _stream())
    return out


def embedding_bwd(dout, ids, dtable, offset=0):
    _lib.call("sat_embedding_bwd", _p(dout), _p(ids), _p(dtable), ids.numel(), dtable.shape[1],
              dtable.shape[0], offset, _stream())


def bn_stats(x2, mean, var, ws, mov_mean=None, mov_var=None, momentum=0.99):
    M, C = x2.shape
    _lib.call("sat_bn_stats", _p(x2), x2.stride(0), M, C, _p(mean), _p(var), _p(mov_mean),
              _p(mov_var), momentum, ws.get(M, C), _stream())


def bn_apply(x2, y2, mean, var, gamma, beta, relu=False, res=None, eps=1e-3):
    M, C = x2.shape
    _lib.call("sat_bn_apply", _p(x2), x2.stride(0), _p(y2), y2.stride(0), M, C, _p(mean),
              _p(var), eps, _p(gamma), _p(beta), int(relu), _p(res), _rs(res), _stream())


def bn_bwd(dy2, x2, gate2, dx2, mean, var, gamma, dgamma, dbeta, ws, training=True,
           beta_out=0.0, eps=1e-3):
    M, C = x2.shape
    _lib.call("sat_bn_bwd", _p(dy2), dy2.stride(0), _p(x2), x2.stride(0), _p(gate2),
              _rs(gate2), _p(dx2), dx2.stride(0), M, C, _p(mean), _p(var), eps, _p(gamma),
              _p(dgamma), _p(dbeta), int(training), beta_out, ws.get(M, C), _stream())


def colsum(x2, out, ws, beta=1.0):
    M, C = x2.shape
    _lib.call("sat_colsum", _p(x2), x2.stride(0), M, C, _p(out), beta, ws.get(M, C), _stream())


def colsum_scatter(x2, dsts, ws, beta=1.0):
    """Column sums of x2 [M, C] split over consecutive destinations (1-D views whose lengths
    add up to at most C): dst = beta * dst + its columns' sums, ONE reduction for all."""
    M, C = x2.shape
    segs = (_lib.SatColSegment * len(dsts))()
    col = 0
    for k, d in enumerate(dsts):
        if not d.is_contiguous():
            raise ValueError("colsum_scatter: destinations must be contiguous")
        segs[k].dst, segs[k].col, segs[k].n = _p(d), col, d.numel()
        col += d.numel()
    _lib.call("sat_colsum_scatter", _p(x2), x2.stride(0), M, C, segs, len(dsts), beta,
              ws.get(M, C), _stream())


def maxpool2(x, y):
    B, N, C = x.shape
    _lib.call("sat_maxpool2", _p(x), _p(y), B, N, C, _stream())
    return y


def bn_apply_maxpool2(x, y, mp, mean, var, gamma, beta, relu=True, eps=1e-3):
    """y = BN(x) (+ReLU) and mp = maxpool2(y) in one pass (x, y, mp [B, N, C] contiguous):
    bit-identical to bn_apply + maxpool2 (sat_bn_apply_maxpool2)."""
    B, N, C = x.shape
    _lib.call("sat_bn_apply_maxpool2", _p(x), _p(y), _p(mp), B, N, C, _p(mean), _p(var), eps,
              _p(gamma), _p(beta), int(relu), _stream())
    return mp


def maxpool2_bwd(x, dy, dx):
    B, N, C = x.shape
    _lib.call("sat_maxpool2_bwd", _p(x), _p(dy), _p(dx), B, N, C, _stream())
    return dx


def highway_fwd(h, t, x, y):
    _lib.call("sat_highway_fwd", _p(h), _p(t), _p(x), _p(y), y.numel(), _stream())
    return y


def highway_act_fwd(h, t, x, y):
    _lib.call("sat_highway_act_fwd", _p(h), _p(t), _p(x), _p(y), y.numel(), _stream())
    return y


def pair_view(a: torch.Tensor, b: torch.Tensor):
    """Two equally shaped contiguous views of ONE storage as a [2, ...] batch view (batch stride
    = their element distance), or None when they cannot be (different storage, overlap).
    Returns (view, swapped): swapped means view[0] is ``b``."""
    if (a.shape != b.shape or not a.is_contiguous() or not b.is_contiguous() or
            a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr()):
        return None
    oa, ob = a.storage_offset(), b.storage_offset()
    swapped = ob < oa
    lo, d = (ob, oa - ob) if swapped else (oa, ob - oa)
    if d < a.numel():
        return None
    base = a if not swapped else b
    full = torch.empty(0, device=a.device, dtype=a.dtype).set_(base.untyped_storage())
    return full.as_strided((2, *a.shape), (d, *a.stride()), lo), swapped


def highway_bwd(h, t, x, dy, dh_pre, dt_pre, dx):
    _lib.call("sat_highway_bwd", _p(h), _p(t), _p(x), _p(dy), _p(dh_pre), _p(dt_pre), _p(dx),
              dy.numel(), _stream())


def act_bwd(dy, y, dx, act, mask=None, beta=0.0):
    _lib.call("sat_act_bwd", _p(dy), _p(y), _p(mask), _p(dx), dy.numel(), ACT[act], beta,
              _stream())
    return dx


def axpby(x, y, a, b):
    _lib.call("sat_axpby", _p(x), _p(y), x.numel(), a, b, _stream())
    return y


def _causal_rows(x, Lq, causal, what):
    """Rows per square matrix for the causal limit: explicit ``Lq``, else x's [.., Lq, L] shape
    (a flattened 2-D [R, L] view cannot tell)."""
    if Lq is not None:
        return int(Lq)
    if causal and x.dim() < 3:
        raise ValueError(f"{what}: causal on a 2-D view needs Lq (rows per [Lq, L] matrix)")
    return x.shape[-2]


def softmax_fwd(S, P, Pd=None, mask=None, causal=False, scale=1.0, Lq=None):
    L = S.shape[-1]
    Lq = _causal_rows(S, Lq, causal, "softmax_fwd")
    R = S.numel() // L
    _lib.call("sat_softmax_fwd", _p(S), _p(P), _p(Pd), _p(mask), R, L, Lq, int(causal), scale,
              _stream())


def softmax_bwd(P, dPd, dS, mask=None, scale=1.0, causal=False, Lq=None):
    L = P.shape[-1]
    Lq = _causal_rows(P, Lq, causal, "softmax_bwd")
    _lib.call("sat_softmax_bwd", _p(P), _p(dPd), _p(mask), _p(dS), P.numel() // L, L,
              Lq, int(causal), scale, _stream())


def loss_fwd_bwd(mel, tgt, tmask, stop, done, dmask, out, dmel=None, dstop=None, l1_weight=0.1):
    B, T, M = mel.shape
    Tp = stop.shape[1]
    ws = _stream_scratch(mel.device, "loss", int(_lib.load().sat_workspace_loss()))
    _lib.call("sat_loss_fwd_bwd", _p(mel), _p(tgt), _p(tmask), _p(stop), _p(done), _p(dmask),
              B, T, M, Tp, l1_weight, _p(out), _p(dmel), _p(dstop), ws, _stream())


def transpose(x: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    R, C = x.shape
    if out is None:
        out = torch.empty(C, R, device=x.device)
    _lib.call("sat_transpose", _p(x), x.stride(0), _p(out), out.stride(0), R, C, _stream())
    return out


# the fused causal attention (sat_flash_attn_fwd/bwd) for the decoder head's shape;
# SAT_FLASH_ATTN=0 keeps the materialised scores (A/B and tests)
FLASH_ATTN = os.environ.get("SAT_FLASH_ATTN", "1") != "0"
# SAT_FLASH_NARROW=0 keeps the encoder's narrow heads on the materialised path (A/B)
FLASH_NARROW = os.environ.get("SAT_FLASH_NARROW", "1") != "0"


def flash_attn_ok(causal: bool, dh: int, L: int) -> bool:
    """the fused attention's two shapes: the decoder head (causal, dh = 128) and narrow heads
    (dh in {8, 16, 32}, L <= 256, causal or not: the encoder's self-attention)"""
    if not FLASH_ATTN:
        return False
    if causal and dh == 128 and L % 4 == 0:
        return True
    return FLASH_NARROW and dh in (8, 16, 32) and L <= 256 and (2 * L * dh + 2 * L) * 4 <= 65536


def flash_attn(q, k, v, o, lse, heads: int, mask=None, dout=None, dq=None, dk=None, dv=None,
               delta=None, causal: bool = True):
    """sat_flash_attn_fwd (dout is None) / _bwd on [B, L, heads*dh] row-major q/k/v/o (the
    backward writes dq, dk, dv; ``delta`` [B, heads, L] scratch, dh = 128 only)."""
    B, L, D = q.shape
    a = _lib.SatFlashAttn()
    a.B, a.H, a.L, a.dh, a.scale, a.ld = B, heads, L, D // heads, 0.0, q.stride(1)
    a.causal = 1 if causal else 0
    a.q, a.k, a.v, a.mask, a.o, a.lse = _p(q), _p(k), _p(v), _p(mask), _p(o), _p(lse)
    if dout is None:
        _lib.check(_lib.load().sat_flash_attn_fwd(ctypes.byref(a), _stream()), "sat_flash_attn_fwd")
        return
    a.dout, a.delta, a.dq, a.dk, a.dv = _p(dout), _p(delta), _p(dq), _p(dk), _p(dv)
    _lib.check(_lib.load().sat_flash_attn_bwd(ctypes.byref(a), _stream()), "sat_flash_attn_bwd")


def mha_desc(x, Wq, bq, Wk, bk, Wv, bv, Wo, bo, heads: int, causal: bool, probs_mask, saved):
    """SatMha over x [B, L, W] with the forward's saved tensors (dict of q, k, v, P, Pd, o, y)."""
    B, L, W = x.shape
    assert x.is_contiguous()
    d = _lib.SatMha()
    d.B, d.L, d.W, d.D, d.H, d.causal = B, L, W, Wq.shape[1], heads, int(causal)
    d.out_dim = Wo.shape[1]
    d.x, d.Wq, d.bq, d.Wk, d.bk = _p(x), _p(Wq), _p(bq), _p(Wk), _p(bk)
    d.Wv, d.bv, d.Wo, d.bo = _p(Wv), _p(bv), _p(Wo), _p(bo)
    d.probs_mask = _p(probs_mask)
    for f in ("q", "k", "v", "P", "Pd", "o", "y", "lse"):
        setattr(d, f, _p(saved.get(f)))
    # the fused path (saved["lse"]: model.mha_fwd chose it under the library's flash_ok rule)
    # needs no [B][H][L][L] score slab in either direction
    size = (_lib.load().sat_mha_scratch_bytes_fused if saved.get("lse") is not None
            else _lib.load().sat_mha_scratch_bytes)
    nbytes = int(size(B, L, d.D, heads, d.out_dim))
    scratch = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
    d.scratch, d.scratch_bytes = scratch.data_ptr(), nbytes
    ws = _gemm_ws(x.device)
    d.gemm_ws, d.gemm_ws_bytes = ws.data_ptr(), ws.numel()
    return d, scratch


def mha_fwd(d):
    _lib.check(_lib.load().sat_mha_fwd(ctypes.byref(d), _stream()), "sat_mha_fwd")


def mha_bwd(d):
    _lib.check(_lib.load().sat_mha_bwd(ctypes.byref(d), _stream()), "sat_mha_bwd")


def mha_bwd_wgrad(d):
    """the four projections' weight / bias gradients a weight-deferred mha_bwd left for later"""
    _lib.check(_lib.load().sat_mha_bwd_wgrad(ctypes.byref(d), _stream()), "sat_mha_bwd_wgrad")
