"""Copy the judged parts of a tools/profile.sh run into profiles/ (tracked):

  profiles/<name>_kernel_stats.csv   rocprofv3 --stats summary of the bench
                                     command
  profiles/<name>_bench.json         the bench line printed under rocprofv3
  profiles/<name>_summary.json       tools/pmc_summary.py output
  profiles/pmc_latest.json           HBM traffic per spec launch, read by
                                     bench.py for roofline.traffic

usage: python tools/keep_profile.py gpurun_out/prof_<tag> <name>
"""
import json
import os
import shutil
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    src, name = sys.argv[1], sys.argv[2]
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, name + "_kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, name + "_bench.json"))
    with open(os.path.join(src, "summary.json")) as f:
        summ = json.load(f)
    with open(os.path.join(dst, name + "_summary.json"), "w") as f:
        json.dump(summ, f, indent=1, sort_keys=True)
        f.write("\n")
    cfg = summ["bench"]["config"]
    t = summ["traffic"]
    latest = {"workload": cfg["workload_id"], "mix": cfg["profile_mix"],
              "chunk": cfg["chunk"], "warmup_eblocks": cfg["warmup_eblocks"],
              "hbm_bytes_per_launch": t["hbm_bytes_per_launch"],
              "read_bytes": t["read_bytes"], "write_bytes": t["write_bytes"],
              "bytes_per_rdreq": t["bytes_per_rdreq"],
              "alg_bytes_per_launch": t["alg_bytes_per_launch"],
              "traffic_over_alg": t["traffic_over_alg"],
              "read_over_xa": t.get("read_over_xa"), "read_over_xa_w0": t.get("read_over_xa_w0"),
              "spec_kernel_us_trace": summ["kernel_us"].get(summ["spec_key"]),
              "spec_kernel_us_trace_alone": summ.get("kernel_us_alone", {}).get(summ["spec_key"]),
              "method": "write = WRITE_SIZE x 1 KiB; read = TCC_EA0_RDREQ x 128 B (one "
                        "request is one 128-B line: tools/rdreq_calib.hip, "
                        "profiles/r03_rdreq_calib.json); per spec launch, L2->fabric "
                        "requests, Infinity-Cache hits included (tools/pmc_summary.py)",
              "source": "profiles/%s_summary.json" % name}
    with open(os.path.join(dst, "pmc_latest.json"), "w") as f:
        json.dump(latest, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps(latest))


if __name__ == "__main__":
    main()
