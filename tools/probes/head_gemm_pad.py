"""Row-stride probe for the decoder head's score products: the [L, L] score / probability
matrices at row stride L (= 500 floats, rows not 128-B aligned) vs a padded stride (512):
S = Q K^T (writes them), O = P V (reads them as A), dV = P^T dO (reads them transposed), with
HIP events (tools only).  Usage: python tools/probes/head_gemm_pad.py [L] [pad] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import kernels as K  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 500
Lp = int(sys.argv[2]) if len(sys.argv) > 2 else 512
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
B, H, D = 32, 2, 256
dh = D // H
q = torch.randn(B, L, D, device="cuda")
k = torch.randn(B, L, D, device="cuda")
Aq = q.view(B, L, H, dh).permute(0, 2, 1, 3)
Bk = k.view(B, L, H, dh).permute(0, 2, 3, 1)
Vv = k.view(B, L, H, dh).permute(0, 2, 1, 3)
O = torch.empty(B, L, D, device="cuda")
Oo = O.view(B, L, H, dh).permute(0, 2, 1, 3)
dV = torch.empty(B, L, D, device="cuda")
dVv = dV.view(B, L, H, dh).permute(0, 2, 1, 3)


def t(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for stride in (L, Lp):
    Sb = torch.empty(B, H, L, stride, device="cuda")
    S = Sb[..., :L]
    P = torch.softmax(torch.randn(B, H, L, L, device="cuda"), -1)
    Pb = torch.zeros(B, H, L, stride, device="cuda")
    Pb[..., :L] = P
    Pv = Pb[..., :L]
    us1 = t(lambda: K.gemm(Aq, Bk, S))
    us2 = t(lambda: K.gemm(Pv, Vv, Oo))
    us3 = t(lambda: K.gemm(Pv.transpose(-1, -2), Oo, dVv))
    print(f"row stride {stride}: S = Q K^T {us1:6.1f} us   O = P V {us2:6.1f} us   "
          f"dV = P^T dO {us3:6.1f} us", flush=True)
