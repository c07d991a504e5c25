"""Overlap of consecutive steps in a pipelined run (bench.py --pipeline D)
from a rocprofv3 kernel trace (tools/trace.sh): per spec launch its
duration, the time it shares with the previous spec launch, and the start
gap after it; the fix kernels' share that runs under a spec launch.

usage: python tools/trace_overlap.py gpurun_out/prof_<tag>
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
    fix = [k for k in ks if "xa_decode_fix" in k[2]]
    dur = [(b - a) / 1e3 for a, b, _ in spec]
    ov = [max(0, spec[i - 1][1] - spec[i][0]) / 1e3 for i in range(1, len(spec))]
    period = [(spec[i][0] - spec[i - 1][0]) / 1e3 for i in range(1, len(spec))]
    hidden = 0.0
    for a, b, _ in fix:
        for c, d, _ in spec:
            hidden += max(0, min(b, d) - max(a, c)) / 1e3
    fix_total = sum((b - a) / 1e3 for a, b, _ in fix)
    m = lambda v: round(sum(v) / len(v), 2) if v else None
    print(json.dumps({"spec_launches": len(spec), "spec_us": m(dur),
                      "spec_overlap_prev_us": m(ov), "spec_start_period_us": m(period),
                      "fix_us": m([(b - a) / 1e3 for a, b, _ in fix]),
                      "fix_under_spec_frac": round(hidden / fix_total, 3) if fix_total else None}))


if __name__ == "__main__":
    main()
