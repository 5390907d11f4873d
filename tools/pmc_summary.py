"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE) for one kernel into per-launch HBM
bytes, with the gfx950 corrections of MI355X_MICROARCH.md (HBM section):
  * FETCH_SIZE and WRITE_SIZE are reported in KiB;
  * FETCH_SIZE counts exactly half the bytes of wide (16 B/lane) coalesced streaming reads on
    gfx950 -> doubled here (the attention kernels' bulk reads are 16-byte float4 loads; other
    widths are uncalibrated, so the doubled figure is an upper estimate for them);
  * WRITE_SIZE is exact for 16-B stores and is taken as is.

    python3 tools/pmc_summary.py <fetch_dir> <write_dir> [kernel_regex [kernel_source.hip]]

With a kernel source file, the summary records its sha256 (first 16 hex digits) so bench.py can
tell whether the committed traffic was measured on the tree it runs.
"""
import hashlib
import glob
import json
import re
import sqlite3
import sys
import csv


def per_dispatch(path, counter, regex):
    vals = []
    csvs = glob.glob(f"{path}/**/*counter_collection.csv", recursive=True)
    if csvs:
        for fn in csvs:
            for r in csv.DictReader(open(fn)):
                if r.get("Counter_Name") == counter and re.search(regex, r.get("Kernel_Name", "")):
                    vals.append(float(r["Counter_Value"]))
        return vals
    for fn in glob.glob(f"{path}/**/*.db", recursive=True):
        db = sqlite3.connect(fn)
        tabs = [t for (t,) in db.execute("select name from sqlite_master where type='table'")]
        pmc = [t for t in tabs if "pmc_event" in t]
        ks = [t for t in tabs if "kernel_symbol" in t]
        kd = [t for t in tabs if "kernel_dispatch" in t]
        info = [t for t in tabs if "info_pmc" in t]
        if not (pmc and ks and kd):
            continue
        q = (f"select e.value, s.kernel_name, i.name from {pmc[0]} e "
             f"join {kd[0]} d on e.event_id = d.event_id "
             f"join {ks[0]} s on d.kernel_id = s.id "
             f"join {info[0]} i on e.pmc_id = i.id")
        try:
            for v, name, cname in db.execute(q):
                if cname == counter and re.search(regex, name):
                    vals.append(float(v))
        except sqlite3.Error as e:
            print("sqlite:", e, file=sys.stderr)
    return vals


def main(fetch_dir, write_dir, regex="attn_energy_kernel", source=None):
    f = per_dispatch(fetch_dir, "FETCH_SIZE", regex)
    w = per_dispatch(write_dir, "WRITE_SIZE", regex)
    out = {"kernel_regex": regex, "dispatches_fetch": len(f), "dispatches_write": len(w)}
    if source:
        out["source"] = source
        out["source_sha16"] = hashlib.sha256(open(source, "rb").read()).hexdigest()[:16]
    if f and w:
        fk = sum(f) / len(f)
        wk = sum(w) / len(w)
        out.update(fetch_kib_raw=fk, write_kib=wk,
                   hbm_bytes_per_launch=int((2 * fk + wk) * 1024),
                   correction="FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
