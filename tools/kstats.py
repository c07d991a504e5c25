"""Median / mean / count of each decode kernel's duration in a rocprofv3
kernel-trace CSV, and for spec -> fix (round 5: tail) pairs the gap between
them and the span from the spec kernel's start to the fix kernel's end:
python3 tools/kstats.py <run_kernel_trace.csv> [label]"""
import collections
import csv
import sys


def main(path, label=""):
    d = collections.defaultdict(list)
    seq = []
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            if "xa_" in n:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                d[n.split("(")[0]].append((e - s) / 1e3)
                seq.append((s, e, "spec" in n, "fix" in n or "tail" in n))
    for n, v in sorted(d.items()):
        v.sort()
        print("%-12s %-40s n=%4d median %8.2f us  mean %8.2f us  min %8.2f" % (
            label, n[:40], len(v), v[len(v) // 2], sum(v) / len(v), v[0]))
    seq.sort()
    gap, span = [], []
    for a, b in zip(seq, seq[1:]):
        if a[2] and b[3]:
            gap.append((b[0] - a[1]) / 1e3)
            span.append((b[1] - a[0]) / 1e3)
    for name, v in (("spec->fix gap", gap), ("spec start->fix end", span)):
        if v:
            v.sort()
            print("%-12s %-40s n=%4d median %8.2f us  mean %8.2f us  min %8.2f" % (
                label, name, len(v), v[len(v) // 2], sum(v) / len(v), v[0]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
