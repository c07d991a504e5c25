"""Per-kernel resource usage of a .hip file (hipcc -Rpass-analysis):
name, VGPRs, AGPRs, scratch bytes/lane, occupancy, LDS bytes.

usage: python tools/kres.py bjxa_amd/csrc/xa_decode.hip [filter]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.dirname(os.path.abspath(src)),
           "-munsafe-fp-atomics", "-c", "-o", "/dev/null", src,
           "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur, rows = None, []
    for ln in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", ln)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        if filt not in r["name"]:
            continue
        dem = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        print("%-62s V%-4s A%-3s scr%-4s occ%-2s lds%s" % (
            dem[:62], r.get("VGPRs", "?"), r.get("AGPRs", "?"),
            r.get("ScratchSize [bytes/lane]", "?"), r.get("Occupancy [waves/SIMD]", "?"),
            r.get("LDS Size [bytes/block]", "?")))


if __name__ == "__main__":
    main()
