#!/bin/bash
# Bytes per L2->fabric read request on known byte counts (GPU box), then
# K1 itself on C3 at warm-up 8 and 0, with the same counters.  One counter
# group per rocprofv3 pass, no trace domains.
#   usage: tools/rdreq_calib.sh <tag>
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/rdcal_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
G1="TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum"
G2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
B="--steps 3 --warmup 1 --no-cpu --no-verify --no-other --chunk 40"
i=0
for grp in "$G1" "$G2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/probe$i" -o run \
      -- "$R/tools/bin/rdreq_calib" > "$OUT/probe$i.log" 2>&1
  for W in 8 0; do
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/k1w${W}_$i" -o run \
        -- python3 "$R/bench.py" $B --warm-blocks $W > "$OUT/k1w${W}_$i.log" 2>&1
  done
done
echo "rdreq calib $TAG done"
