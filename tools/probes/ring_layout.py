"""Driver of ring_layout_skeleton.hip (tools only): per-step cost of the attention forward's two
hand-offs + LDS phases in the built layout (8 workgroups x 8 waves per utterance, one per CU)
against 16 workgroups x 4 waves per utterance with two utterances co-resident per CU, at equal
per-CU dummy compute."""
import ctypes
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
src = os.path.join(HERE, "ring_layout_skeleton.hip")
so = os.path.join(HERE, "ring_layout_skeleton.so")
if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    "-I" + os.path.join(HERE, "../../include"), src, "-o", so], check=True)
lib = ctypes.CDLL(so)
dev = torch.device("cuda")
cus = torch.cuda.get_device_properties(0).multi_processor_count
T = 500
names = {0: "8 WG x 8 waves / utterance", 1: "16 WG x 4 waves, 2 per CU"}
for layout in (0, 1):
    occ = lib.ring_layout_occupancy(layout)
    need = 1 if layout == 0 else 2
    if occ * cus < 256 * need:
        print(f"{names[layout]}: not co-resident ({occ} per CU x {cus} CUs); skipped", flush=True)
        continue
    for nbar in (0, 4):
        for crit in (0, 50, 150):
            RA = torch.zeros(2 * 32 * 2048, device=dev)
            RB = torch.zeros_like(RA)
            err = torch.zeros(2, dtype=torch.int32, device=dev)
            clk = torch.zeros(512, dtype=torch.int64, device=dev)
            ts = []
            for rep in range(3):
                RA.zero_(); RB.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                lib.ring_layout(layout, ctypes.c_void_p(RA.data_ptr()), ctypes.c_void_p(RB.data_ptr()),
                                T, crit, nbar, 1, ctypes.c_void_p(err.data_ptr()),
                                ctypes.c_void_p(clk.data_ptr()),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                e1.record()
                torch.cuda.synchronize()
                if rep:
                    ts.append(e0.elapsed_time(e1) * 1e3 / T)
            print(f"{names[layout]:28s} nbar={nbar} crit={crit:4d} FMAs/phase: "
                  f"{min(ts):6.3f} us/step (err {int(err[0])})", flush=True)
