#!/bin/bash
# rocprofv3 passes over a short bench run (GPU box).  Kernel trace + stats in
# one pass; each PMC group in its own pass (counters never combined with
# trace domains).  Output under gpurun_out/prof_<tag>/.
#   usage: tools/profile.sh <tag> [bench args...]
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 5 --warmup 1 --no-cpu --no-verify $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU" \
    "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE" \
    "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
    "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run \
      -- python3 "$R/bench.py" $ARGS > "$OUT/pmc$i.log" 2>&1 || echo "pmc pass $i ($grp) failed rc=$?"
done
echo "profile $TAG done"
