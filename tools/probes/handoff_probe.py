"""Driver of handoff_probe.hip (tools only): per-round cost of an in-kernel group barrier with
a 16-B-per-workgroup payload, for group sizes 32 (one XCD under round-robin placement) and 256."""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "handoff_probe.so")
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                os.path.join(HERE, "handoff_probe.hip"), "-o", so], check=True)
lib = ctypes.CDLL(so)


def run(G, W, rounds):
    dev = torch.device("cuda")
    ctr = torch.zeros(32 * G, dtype=torch.int32, device=dev)
    rec = torch.zeros(W, 4, device=dev)
    err = torch.zeros(2, dtype=torch.int32, device=dev)
    clk = torch.zeros(W, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rc = lib.launch_probe(G, W, rounds, ctypes.c_void_p(ctr.data_ptr()),
                          ctypes.c_void_p(rec.data_ptr()), ctypes.c_void_p(err.data_ptr()),
                          ctypes.c_void_p(clk.data_ptr()),
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    e1.record()
    torch.cuda.synchronize()
    assert rc == 0, rc
    ms = e0.elapsed_time(e1)
    print(f"G={G:3d} groups x {W // G:3d} WGs, {rounds} rounds: {1e3 * ms / rounds:7.3f} us/round"
          f"  stale={int(err[0])} timeouts={int(err[1])}", flush=True)


if __name__ == "__main__":
    for G, W in ((8, 256), (1, 256), (8, 64), (32, 256)):
        run(G, W, 2000)
