"""Driver of pingpong.hip (tools only): one-way hand-off latency of a 1-KB tagged record between
two workgroups of one XCD, for the three poll styles."""
import ctypes
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "pingpong.so")
if not os.path.exists(so):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    "-I" + os.path.join(HERE, "../../include"),
                    os.path.join(HERE, "pingpong.hip"), "-o", so], check=True)
lib = ctypes.CDLL(so)
dev = torch.device("cuda")
rounds = 20000
for style, name in [(0, "load/wait/sleep1"), (2, "two in flight")]:
    for rep in range(2):
        buf = torch.zeros(4 * 64 * 4, device=dev)
        out = torch.zeros(2, dtype=torch.int64, device=dev)
        xcc = torch.zeros(2, dtype=torch.int32, device=dev)
        rc = lib.pingpong(style, ctypes.c_void_p(buf.data_ptr()), rounds,
                          ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(xcc.data_ptr()),
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        ticks = int(out[0])
        print(f"style {style} {name:18s} rep {rep}: {ticks * 10.0 / rounds / 2:7.1f} ns one-way "
              f"(xcc {xcc.tolist()}, rc {rc})", flush=True)

