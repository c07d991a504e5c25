"""Per-step timeline of the decode from a rocprofv3 kernel trace
(tools/trace.sh): mean duration of each kernel and of the idle gaps
spec -> fix and fix -> next spec, in microseconds.

usage: python tools/trace_gaps.py gpurun_out/prof_<tag>
"""
import csv
import glob
import json
import os
import sys


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "trace", "**", "*kernel_trace.csv"),
                       recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                 for r in rows), key=lambda x: x[0])
    spec = [k for k in ks if "xa_decode_spec" in k[2]]
    out = {"spec_us": [], "fix_us": [], "gap_spec_fix_us": [], "gap_fix_spec_us": []}
    for i, k in enumerate(ks):
        if "xa_decode_spec" in k[2] and i + 1 < len(ks) and "xa_decode_fix" in ks[i + 1][2]:
            f = ks[i + 1]
            out["spec_us"].append((k[1] - k[0]) / 1e3)
            out["fix_us"].append((f[1] - f[0]) / 1e3)
            out["gap_spec_fix_us"].append((f[0] - k[1]) / 1e3)
            if i + 2 < len(ks) and "xa_decode_spec" in ks[i + 2][2]:
                out["gap_fix_spec_us"].append((ks[i + 2][0] - f[1]) / 1e3)
    print(json.dumps({k: round(sum(v) / len(v), 2) if v else None for k, v in out.items()} |
                     {"steps": len(out["spec_us"]), "spec_launches": len(spec)}))


if __name__ == "__main__":
    main()
