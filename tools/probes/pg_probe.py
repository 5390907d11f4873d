"""Isolated timing of sat_attn_param_grads at the C2 shape (T'=500, B=32, N=200): energies
recomputed vs z read from the ZH history.  GPU tool:  python tools/probes/pg_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import _sat_path  # noqa: E402

_sat_path.load()
from sat_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    T, B, N, D1, D2, F, KW = 500, 32, 200, 224, 32, 5, 10
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g)   # noqa: E731
    K1, K2, q = r(B, N, D1), r(B, N, D2), r(T, B, D1 + D2)
    b1, v1, v2, locW = r(D1), r(D1), r(D2), r(F, D1)
    loc, sp, de1, de2, df = r(T, B, N, F), r(T, B, N), r(T, B, N), r(T, B, N), r(T, B, N, F)
    zh = torch.tanh(r(T, B, N, D1 + D2))
    pgs = K.pg_stride(D1, D2, F, KW)
    PG = torch.empty(K.attn_param_grad_rows(B, N), pgs, device=dev)
    dK1, dK2 = torch.empty(B, N, D1, device=dev), torch.empty(B, N, D2, device=dev)

    def run(z, share):
        K.attn_param_grads(T=T, B=B, N=N, D1=D1, D2=D2, F=F, KW=KW, att1_forward=1, K1=K1, K2=K2,
                           q=q, q_tstride=q.stride(0), q_bstride=q.stride(1), b1=b1, v1=v1,
                           locW=locW, v2=v2, loc=loc, s_prev=sp, s_tstride=sp.stride(0),
                           de1=de1, de2=de2, df=df, dK1=dK1, dK2=dK2, pg=PG, pg_stride=pgs, zh=z,
                           zh_share=share)

    for share in range(9):
        z = zh if share else None
        name = f"zh {share}/8"
        for _ in range(3):
            run(z, share)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run(z, share)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        zb = T * B * N * (D1 + D2) * 4 * share / 8
        print(f"{name:10s} {us:8.1f} us/launch  ZH stream {zb / us / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
