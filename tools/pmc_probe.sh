#!/bin/bash
# Stall-counter passes over the C3 bench (one counter group per rocprofv3
# run, no trace domains): TLB (UTCL1), TA/TD/TCP stalls, L2 write stalls,
# SQ wait breakdown.  Output: gpurun_out/pmcprobe_<tag>/pmc<i>/, then a
# per-kernel mean table (tools/pmc_summary.py counters()).
#   usage: tools/pmc_probe.sh <tag> [bench args...]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmcprobe_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
PM="--steps 5 --warmup 1 --no-cpu --no-verify --no-other"
i=0
for grp in \
    "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
    "TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum GRBM_GUI_ACTIVE" \
    "TA_BUSY_avr TA_TA_BUSY_sum" \
    "TD_TD_BUSY_sum" \
    "TCC_EA0_WRREQ_STALL_sum TCC_BUSY_avr TCC_TAG_STALL_sum" \
    "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run \
      -- python3 "$R/bench.py" "$@" $PM > "$OUT/pmc$i.log" 2>&1 || {
	echo "pmc pass $i ($grp) failed rc=$?"; exit 1; }
done
python3 - "$OUT" <<'PY'
import sys, json
sys.path.insert(0, sys.argv[1] + "/../../tools")
from pmc_summary import counters
c = counters(sys.argv[1] + "/pmc*/**/*counter_collection.csv")
print(json.dumps({k: v for k, v in c.items() if "spec" in k or "fix" in k}, indent=1))
PY
