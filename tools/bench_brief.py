"""One-screen summary of a bench.py JSON line (the last line of the file):
usage: python tools/bench_brief.py <bench.json>"""
import json
import sys


def main(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print("%s n=%s value=%s ms/step=%s serial=%s spread=%s launch_ms=%s frac=%s step_frac=%s "
          "exact=%s" % (d["config"].get("workload_id", d["config"].get("workload")),
                        d["n_gpus"], d["value"], d["ms_per_step"], d.get("ms_per_step_serial"),
                        d.get("step_ms"), r.get("launch_ms"), r.get("frac"), r.get("step_frac"),
                        d.get("bit_exact")))
    for k, v in (d.get("other_configs") or {}).items():
        print("  %-9s ms/step=%s serial=%s kernel_ms=%s frac=%s exact=%s" % (
            k, v.get("ms_per_step"), v.get("ms_per_step_serial"),
            v.get("spec_ms", v.get("kernel_ms")), v.get("frac"), v.get("bit_exact")))


if __name__ == "__main__":
    main(sys.argv[1])
