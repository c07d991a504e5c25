"""Per-kernel mean of each counter in a rocprofv3 --pmc CSV directory, with
TCC_EA0_RDREQ / WRREQ turned into bytes (128 B per read request,
profiles/r03_rdreq_calib.json; 64 B per write request):
python3 tools/pmc_brief.py <dir> [label]"""
import collections
import csv
import glob
import sys


def main(d, label=""):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                n = r["Kernel_Name"]
                if "xa_" in n:
                    acc[n.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, cs in sorted(acc.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        rd = m.get("TCC_EA0_RDREQ_sum", 0) * 128 / 1e6
        wr = m.get("TCC_EA0_WRREQ_sum", 0) * 64 / 1e6
        print("%-12s %-40s read %8.1f MB  write %8.1f MB  (n=%d)" % (
            label, n[:40], rd, wr, len(next(iter(cs.values())))))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
