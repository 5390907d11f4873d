"""Dynamic instruction mix of the persistent decoder kernels from one rocprofv3 PMC pass
(tools only; run on the GPU box from the repo root):

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS \
        SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace -d <dir> -o pmc \
        -- python3 tools/pmc_persistent.py
    python3 tools/pmc_instmix.py <dir> <kernel_regex> <steps per launch> [source.hip]

Per launch, per wave and per decoder step (counts are summed over every wave of the launch by
the hardware): VALU, SALU, branch, LDS, scalar-memory and vector-memory instructions, and the
ratio (SALU + branch) / VALU -- the executed counterpart of the static census of
tools/isa_phases.py (both sides of a role branch counted there, only the taken path here).
"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import per_dispatch  # noqa: E402

COUNTERS = ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS",
            "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR")


def main(path, regex, steps, source=None):
    steps = int(steps)
    out = {"kernel_regex": regex, "steps_per_launch": steps}
    if source:
        out["source"] = source
        out["source_sha16"] = hashlib.sha256(open(source, "rb").read()).hexdigest()[:16]
    avg = {}
    for c in COUNTERS:
        v = per_dispatch(path, c, regex)
        if v:
            avg[c] = sum(v) / len(v)
            out.setdefault("dispatches", len(v))
    out["per_launch"] = avg
    waves = avg.get("SQ_WAVES")
    if waves:
        out["per_wave_per_step"] = {c[len("SQ_INSTS_"):].lower(): round(v / waves / steps, 1)
                                    for c, v in avg.items() if c.startswith("SQ_INSTS_")}
    valu = avg.get("SQ_INSTS_VALU")
    if valu:
        out["salu_plus_branch_over_valu"] = round(
            (avg.get("SQ_INSTS_SALU", 0.0) + avg.get("SQ_INSTS_BRANCH", 0.0)) / valu, 3)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:])
