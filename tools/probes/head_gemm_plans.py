"""The decoder head's per-(utterance, head) score products at the step's shape (B*H = 64 matrices
of L x L from [L, dh] operands with row stride D = 256): HIP-event time of each forced LDS plan
(tile / no split) vs the planner's pick, plain and with the causal hint (tools only).
Usage: python tools/probes/head_gemm_plans.py [L] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import _lib  # noqa: E402
from sat_amd import kernels as K  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 500
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
B, H, D = 32, 2, 256
dh = D // H
q = torch.randn(B, L, D, device="cuda")
k = torch.randn(B, L, D, device="cuda")
S = torch.empty(B, H, L, L, device="cuda")
P = torch.softmax(torch.randn(B, H, L, L, device="cuda"), -1)
O = torch.empty(B, L, D, device="cuda")
# views: A [B, H, L, dh] (head slices of the [B, L, D] rows), B = K^T per head
Aq = q.view(B, L, H, dh).permute(0, 2, 1, 3)
Bk = k.view(B, L, H, dh).permute(0, 2, 3, 1)
Vv = k.view(B, L, H, dh).permute(0, 2, 1, 3)
Oo = O.view(B, L, H, dh).permute(0, 2, 1, 3)


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


lib = _lib.load()
for plan in [(0, 0), (128, 64), (64, 128), (64, 64), (128, 128)]:
    lib.sat_gemm_force_plan(plan[0], plan[1], 1)
    for tri in (0, 1):
        us = t(lambda: K.gemm(Aq, Bk, S, tri=tri))
        print(f"S = Q K^T  plan {plan} tri {tri}: {us:7.1f} us", flush=True)
    for tri in (0, 2):
        us = t(lambda: K.gemm(P, Vv, Oo, tri=tri))
        print(f"O = P V    plan {plan} tri {tri}: {us:7.1f} us", flush=True)
lib.sat_gemm_force_plan(0, 0, 0)
