"""Summarise tools/profile.sh output.

usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [--json out.json]

  kernel_us      per-kernel mean duration from the kernel trace of the bench
  kernel_us_alone  the same over launches that overlap no other kernel (the
                 serial event pass of a pipelined bench run)
                 command (trace/), and kernel_n the dispatch counts
  pmc            per-kernel, per-dispatch mean of every counter (pmc*/)
  traffic        HBM bytes per xa_decode_spec launch:
                   write = WRITE_SIZE x 1 KiB (MI355X_MICROARCH.md §HBM: exact
                           for 16-B/lane streaming stores, which these are)
                   read  = TCC_EA0_RDREQ x 128 B: one request is one 128-B
                           line, measured on known byte counts with the
                           decode's own load forms (tools/rdreq_calib.hip,
                           profiles/r03_rdreq_calib.json; TCC_BUBBLE reads 0,
                           so FETCH_SIZE counts each as 64 B -- the guide's
                           x2).  The warm-up-0 pass (pmc_w0/) gives the
                           pattern's own overfetch (read / XA bytes with no
                           warm-up re-read).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


RDREQ_BYTES = 128      # profiles/r03_rdreq_calib.json


def rows(pattern):
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def short(name):
    """Kernel key: name plus <bits,ch> for the templated kernels, so the
    C3 (8-bit stereo) and C2 (8-bit mono) launches of one run stay apart."""
    for k in ("xa_decode_spec", "xa_decode_tail", "xa_decode_fix", "xa_encode_waves",
              "xa_ws_init"):
        if k in name:
            i = name.find(k + "<")
            if i >= 0:
                inner = name[i + len(k) + 1:name.find(">", i)]
                args = [x.strip() for x in inner.split(",")]
                return "%s<%s,%s>" % (k, args[0], args[1])
            return k
    return name[:40]


def counters(pattern):
    pmc = defaultdict(lambda: defaultdict(list))
    for r in rows(pattern):
        pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in pmc.items()}


def main():
    d = sys.argv[1]
    out = {}
    bench = None
    bj = os.path.join(d, "bench.json")
    if os.path.exists(bj):
        lines = [ln for ln in open(bj).read().splitlines() if ln.startswith("{")]
        if lines:
            bench = json.loads(lines[-1])
            out["bench"] = bench
    dur = defaultdict(list)
    ks = []
    for r in rows(os.path.join(d, "trace", "**", "*kernel_trace.csv")):
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[short(r["Kernel_Name"])].append(b - a)
        ks.append((a, b, short(r["Kernel_Name"])))
    out["kernel_us"] = {k: round(sum(v) / len(v) / 1e3, 2) for k, v in dur.items()}
    out["kernel_n"] = {k: len(v) for k, v in dur.items()}
    # launches that share no time with any other kernel: with bench.py's
    # --pipeline > 1 the timed steps overlap, and only the serial event pass
    # (whose median is roofline.launch_ms) runs each kernel alone
    ks.sort()
    alone = defaultdict(list)
    for i, (a, b, k) in enumerate(ks):
        prev_end = max((e for _, e, _ in ks[:i]), default=0)
        nxt = ks[i + 1][0] if i + 1 < len(ks) else b + 1
        if prev_end <= a and nxt >= b:
            alone[k].append(b - a)
    out["kernel_us_alone"] = {k: round(sum(v) / len(v) / 1e3, 2) for k, v in alone.items()}
    out["kernel_n_alone"] = {k: len(v) for k, v in alone.items()}
    out["pmc"] = counters(os.path.join(d, "pmc[0-9]*", "**", "*counter_collection.csv"))
    w0 = counters(os.path.join(d, "pmc_w0", "**", "*counter_collection.csv"))
    out["pmc_w0"] = w0
    cfg = bench["config"] if bench else None
    key = "xa_decode_spec<%d,%d>" % (cfg["bits"], cfg["channels"]) if cfg else ""
    out["spec_key"] = key
    sp = out["pmc"].get(key, {})
    if bench and "TCC_EA0_RDREQ_sum" in sp and "TCC_EA0_RDREQ_sum" in w0.get(key, {}):
        xa_bytes = cfg["eblocks_per_rank"] * cfg["channels"] * (cfg["bits"] * 4 + 1)
        bpr = RDREQ_BYTES
        read = sp["TCC_EA0_RDREQ_sum"] * bpr
        write = sp.get("WRITE_SIZE", 0.0) * 1024
        t = {"read_bytes": round(read), "write_bytes": round(write),
             "hbm_bytes_per_launch": round(read + write),
             "bytes_per_rdreq": bpr,
             "read_over_xa": round(read / xa_bytes, 4),
             "read_over_xa_w0": round(w0[key]["TCC_EA0_RDREQ_sum"] * bpr / xa_bytes, 4),
             "alg_bytes_per_launch": xa_bytes + cfg["eblocks_per_rank"] * 64 * cfg["channels"]}
        if "FETCH_SIZE" in sp:
            t["fetch_size_raw_bytes"] = round(sp["FETCH_SIZE"] * 1024)
            t["fetch_size_x2_bytes"] = round(sp["FETCH_SIZE"] * 2048)
        t["traffic_over_alg"] = round(t["hbm_bytes_per_launch"] / t["alg_bytes_per_launch"], 4)
        out["traffic"] = t
    js = json.dumps(out, indent=1, sort_keys=True)
    print(js)
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
