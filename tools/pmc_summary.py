"""Summarise tools/profile.sh output: per-kernel mean duration (kernel trace)
and per-dispatch mean of every PMC counter for the decode kernels.

usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [--json out.json]
HBM bytes: FETCH_SIZE and WRITE_SIZE are in KiB (x1024).  MI355X_MICROARCH.md
§HBM: on gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide coalesced
streaming read; the raw value is reported and the x2 correction is applied
only where stated.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def short(name):
    for k in ("xa_decode_spec", "xa_decode_fix", "xa_decode_tail", "xa_encode_groups"):
        if k in name:
            return k
    return name[:40]


def main():
    d = sys.argv[1]
    out = {}
    dur = defaultdict(list)
    for r in rows(os.path.join(d, "trace", "**", "*kernel_trace.csv")):
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out["kernel_us"] = {k: round(sum(v) / len(v) / 1e3, 2) for k, v in dur.items()}
    out["kernel_n"] = {k: len(v) for k, v in dur.items()}
    pmc = defaultdict(lambda: defaultdict(list))
    for r in rows(os.path.join(d, "pmc*", "**", "*counter_collection.csv")):
        pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out["pmc"] = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in pmc.items()}
    sp = out["pmc"].get("xa_decode_spec", {})
    if "FETCH_SIZE" in sp and "WRITE_SIZE" in sp:
        out["spec_fetch_bytes_raw"] = sp["FETCH_SIZE"] * 1024
        out["spec_write_bytes"] = sp["WRITE_SIZE"] * 1024
    js = json.dumps(out, indent=1, sort_keys=True)
    print(js)
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            f.write(js)


if __name__ == "__main__":
    main()
