"""Per-kernel medians of every counter in rocprofv3 --pmc CSVs.

usage: python tools/pmc_table.py <dir-or-glob>... [--filter substr]
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = ""
    if "--filter" in sys.argv:
        filt = sys.argv[sys.argv.index("--filter") + 1]
        args = [a for a in args if a != filt]
    files = []
    for a in args:
        files += glob.glob(os.path.join(a, "**", "*counter_collection.csv"), recursive=True) \
            if os.path.isdir(a) else glob.glob(a)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(files):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            per[(r["Dispatch_Id"], r["Kernel_Name"])][r["Counter_Name"]] = float(r["Counter_Value"])
        for (_, k), c in per.items():
            name = k.split("(")[0].replace("void ", "")
            if filt and filt not in name:
                continue
            for n, v in c.items():
                agg[name][n].append(v)
    for k, c in agg.items():
        print(k)
        for n, v in sorted(c.items()):
            print("   %-32s %16.0f  (n=%d)" % (n, statistics.median(v), len(v)))


if __name__ == "__main__":
    main()
