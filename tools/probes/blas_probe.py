"""fp32 library GEMM (torch.mm -> hipBLASLt/rocBLAS, TF32 off) on the training step's largest
GEMM shapes, for comparison with sat_gemm (tools/gemm_census.py).  GPU only."""
import torch

torch.backends.cuda.matmul.allow_tf32 = False
shapes = [(256, 1024, 16000), (544, 1024, 16000), (256, 224, 16000), (256, 256, 16000),
          (16000, 288, 1024), (256, 32, 16000), (16000, 256, 256), (16000, 1024, 288),
          (16000, 256, 1024), (16000, 1024, 256), (6400, 128, 6144), (6400, 2048, 384),
          (128, 128, 6400), (6400, 128, 2048)]
for M, N, K in shapes:
    for ta in (False, True):
        a = torch.randn(K, M, device="cuda").t() if ta else torch.randn(M, K, device="cuda")
        b = torch.randn(K, N, device="cuda")
        c = torch.empty(M, N, device="cuda")
        for _ in range(3):
            torch.mm(a, b, out=c)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            torch.mm(a, b, out=c)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"M={M:6d} N={N:5d} K={K:6d} At={int(ta)}  {us:8.1f} us  {2*M*N*K/us/1e6:6.1f} TF/s", flush=True)
