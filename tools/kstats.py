"""Median / mean / count of each decode kernel's duration in a rocprofv3
kernel-trace CSV: python3 tools/kstats.py <run_kernel_trace.csv> [label]"""
import collections
import csv
import sys


def main(path, label=""):
    d = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            if "xa_" in n:
                d[n.split("(")[0]].append((int(r["End_Timestamp"]) -
                                           int(r["Start_Timestamp"])) / 1e3)
    for n, v in sorted(d.items()):
        v.sort()
        print("%-12s %-40s n=%4d median %8.2f us  mean %8.2f us  min %8.2f" % (
            label, n[:40], len(v), v[len(v) // 2], sum(v) / len(v), v[0]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
