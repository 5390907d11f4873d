"""Cost of the materialised dropout mask in the decoder head's fused attention (C2 shape:
B=32, L=T'=500, 2 heads x 128): sat_flash_attn_fwd / _bwd timed with the [B][H][L][L] probability
mask and without one (tools only, GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
import torch  # noqa: E402

from sat_amd import kernels as K  # noqa: E402

B, L, H, dh = 32, 500, 2, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v, dout = (torch.randn(B, L, H * dh, device="cuda", generator=g) * 0.3 for _ in range(4))
o = torch.empty_like(q)
lse = torch.empty(B, H, L, device="cuda")
delta = torch.empty(B, H, L, device="cuda")
dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
mask = (torch.rand(B, H, L, L, device="cuda", generator=g) < 0.9).float() / 0.9


def t_of(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


for m, name in ((mask, "mask"), (None, "no mask")):
    tf = t_of(lambda: K.flash_attn(q, k, v, o, lse, H, mask=m))
    tb = t_of(lambda: K.flash_attn(q, k, v, o, lse, H, mask=m, dout=dout, dq=dq, dk=dk, dv=dv,
                                   delta=delta))
    print(f"{name:8s} fwd {tf:7.1f} us  bwd (delta + both roles) {tb:7.1f} us", flush=True)
