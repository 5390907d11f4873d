"""Which library kernels torch.mm (hipBLASLt / rocBLAS, fp32, TF32 off) picks for the step's
large-M GEMM shapes -- run under rocprofv3 --kernel-trace --stats to read the kernel names
(macro tile, depth, MFMA shape) next to their times (tools only, GPU)."""
import torch

torch.backends.cuda.matmul.allow_tf32 = False
for M, N, K in [(16000, 1024, 256), (16000, 1024, 544), (16000, 256, 1024), (16000, 1024, 1024)]:
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda")
    c = torch.empty(M, N, device="cuda")
    for _ in range(10):
        torch.mm(a, b, out=c)
    torch.cuda.synchronize()
    print(M, N, K, flush=True)
