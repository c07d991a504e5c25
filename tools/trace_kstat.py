"""Mean and median duration per decode kernel from rocprofv3 trace
databases (the default rocpd output), e.g. of tools/ab_libs.sh runs.

usage: python3 tools/trace_kstat.py 'gpurun_out/ab_*/run_results.db'
"""
import collections
import glob
import sqlite3
import sys


def main():
    for f in sorted(glob.glob(sys.argv[1])):
        c = sqlite3.connect(f)
        d = collections.defaultdict(list)
        for n, dur in c.execute("select name, duration from kernels"):
            d[n].append(dur)
        for n, v in d.items():
            if "xa_" in n:
                v = sorted(v)
                print("%-24s %-44s %4d mean %8.2f us  median %8.2f us" % (
                    f.split("/")[-2], n[:44], len(v), sum(v) / len(v) / 1e3,
                    v[len(v) // 2] / 1e3))


if __name__ == "__main__":
    main()
