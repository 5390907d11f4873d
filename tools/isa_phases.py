"""Instruction census of a persistent kernel's step loop, split at its s_barrier
instructions (the phases of one decoder step), from the gfx950 assembly (hipcc -S).

    python3 tools/isa_phases.py kernel.s <kernel-symbol-substring> [first_line last_line]

For each barrier-delimited region: instruction counts by class (VALU, packed FMA,
transcendental, DPP / permlane cross-lane, LDS, global / buffer memory, scalar, waitcnt,
MFMA, branches) -- the raw material of the critical-path account in DESIGN.md section 5.
Counts are static (both sides of a role branch are counted), so per-wave paths are read
from the region's basic blocks when the roles differ."""
import re
import sys


def classify(op, line):
    if op.startswith("v_mfma"):
        return "mfma"
    if op in ("v_exp_f32", "v_rcp_f32", "v_log_f32", "v_sqrt_f32", "v_rsq_f32", "v_sin_f32",
              "v_cos_f32", "v_rcp_iflag_f32"):
        return "trans"
    if op.startswith("v_permlane") or "row_" in line or "quad_perm" in line or "row_bcast" in line \
            or op.startswith("v_readlane") or op.startswith("v_readfirstlane") or \
            op.startswith("v_writelane") or op.startswith("ds_swizzle") or op.startswith("ds_bpermute"):
        return "xlane"
    if op.startswith("v_pk_fma") or op.startswith("v_pk_mul") or op.startswith("v_pk_add"):
        return "pk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        return "vmem"
    if op == "s_waitcnt":
        return "wait"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path, sym, lo=None, hi=None):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) or
                 (l.rstrip().endswith(":") and sym in l and not l.startswith("\t")))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or
               lines[i].startswith(".Lfunc_end"))
    lo = int(lo) if lo else start
    hi = int(hi) if hi else end
    regions, cur, first = [], {}, lo
    for i in range(lo, hi):
        l = lines[i].strip()
        if not l or l.startswith(";") or l.startswith(".") or l.endswith(":"):
            continue
        op = re.sub(r"_(e32|e64|sdwa|dpp)$", "", l.split()[0])
        c = classify(op, l)
        cur[c] = cur.get(c, 0) + 1
        if op == "s_barrier":
            regions.append((first + 1, i + 1, cur))
            cur, first = {}, i + 1
    regions.append((first + 1, hi, cur))
    keys = ["valu", "pk", "trans", "xlane", "lds", "vmem", "mfma", "salu", "wait", "branch"]
    print("lines".ljust(13) + "".join(k.rjust(7) for k in keys))
    for a, b, cnt in regions:
        print(f"{a:5d}-{b:<6d} " + "".join(str(cnt.get(k, 0)).rjust(7) for k in keys))


if __name__ == "__main__":
    main(*sys.argv[1:])
