import os, sys
sys.path.insert(0, os.getcwd())
import _sat_path
_sat_path.load()
import torch
from sat_amd import kernels
cuda = "cuda"
M, N, K1, K2 = 16000, 1024, 256, 288
for tb in (False,):
    g = torch.Generator().manual_seed(M + K2)
    A = torch.randn(M, K1, generator=g)
    wide = torch.randn(M, K2 + 40, generator=g)
    B = torch.randn(N, K1 + K2, generator=g) if tb else torch.randn(K1 + K2, N, generator=g)
    bias = torch.randn(N, generator=g)
    Bd = B.to(cuda); wd = wide.to(cuda)
    C = kernels.gemm(A.to(cuda), Bd.t() if tb else Bd, bias=bias.to(cuda), A2=wd[:, :K2])
    Al = torch.cat([A, wide[:, :K2]], 1).double().to(cuda)
    Bl = (B.t() if tb else B).double().to(cuda)
    ref = Al @ Bl + bias.double().to(cuda)
    mag = Al.abs() @ Bl.abs() + bias.double().abs().to(cuda)
    err = (C.double() - ref).abs()
    r = err / (4e-7 * mag + 1e-7)
    print(os.environ.get("SAT_GEMM_BIG"), "tb", tb, "max err/bound", float(r.max()), "count>1", int((r > 1).sum()),
          "max err/mag", float((err / mag).max()), "mean err/mag", float((err / mag).mean()))
