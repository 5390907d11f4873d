"""Driver of ring8_skeleton.hip (tools only): per-step cost of the attention forward's two
8-producer hand-offs at its geometry, bare and with dummy dependent compute."""
import ctypes
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "ring8_skeleton.so")
if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(os.path.join(HERE, "ring8_skeleton.hip")):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    "-I" + os.path.join(HERE, "../../include"),
                    os.path.join(HERE, "ring8_skeleton.hip"), "-o", so], check=True)
lib = ctypes.CDLL(so)
dev = torch.device("cuda")
T = 500
for xl, pre, nbar in [(1, 0, 0), (0, 0, 0), (1, 0, 3), (1, 0, 4), (1, 0, 8)]:
    for crit, shadow in [(0, 0), (0, 50), (25, 0)]:
        RA = torch.zeros(2 * 32 * 8 * 64 * 4, device=dev)
        RB = torch.zeros_like(RA)
        err = torch.zeros(2, dtype=torch.int32, device=dev)
        clk = torch.zeros(256 + 64 * 2 * 4, dtype=torch.int64, device=dev)
        for rep in range(2):
            RA.zero_(); RB.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            lib.ring8(ctypes.c_void_p(RA.data_ptr()), ctypes.c_void_p(RB.data_ptr()), T, crit, shadow,
                      xl, pre, nbar, ctypes.c_void_p(err.data_ptr()), ctypes.c_void_p(clk.data_ptr()),
                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            e1.record()
            torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3
        inner = float(clk[:256].double().mean()) / 100.0
        ev = clk[256:].view(64, 2, 4).double().cpu()
        evs = " ".join(f"ph{ph}: poll@{float(ev[:, ph, 0].mean()) * 10:5.0f}ns done@{float(ev[:, ph, 1].mean()) * 10:5.0f} "
                       f"bar@{float(ev[:, ph, 2].mean()) * 10:5.0f} spins {float(ev[:, ph, 3].mean()):4.1f}"
                       for ph in range(2))
        print(f"xl={xl} pre={pre} bars/handoff={1 + nbar} crit={crit:4d} shadow={shadow:4d} FMAs/phase: {us / T:6.3f} us/step "
              f"(in-kernel {inner / T:6.3f}), err {int(err[0])} | {evs}", flush=True)
