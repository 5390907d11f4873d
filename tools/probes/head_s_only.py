"""Drive the decoder head's score product S = Q K^T (B*H = 64 matrices of 500 x 500 from
[500, 128] head slices) repeatedly, for rocprofv3 --pmc passes (tools only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import kernels as K  # noqa: E402

B, H, D, L = 32, 2, 256, 500
dh = D // H
q = torch.randn(B, L, D, device="cuda")
k = torch.randn(B, L, D, device="cuda")
S = torch.empty(B, H, L, L, device="cuda")
Aq = q.view(B, L, H, dh).permute(0, 2, 1, 3)
Bk = k.view(B, L, H, dh).permute(0, 2, 3, 1)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    K.gemm(Aq, Bk, S)
torch.cuda.synchronize()
