#!/bin/bash
# rocprofv3 evidence for the bench line (GPU box).  Output under
# gpurun_out/prof_<tag>/:
#   trace/    --kernel-trace --stats of the bench command itself (bench args
#             as given; none = the driver's default `python bench.py`),
#             bench.json = the line that run printed
#   pmc*/     one counter group per pass (counters never combined with trace
#             domains), on a short run of the same workload
#   pmc_w0/   L2->HBM read requests with warm-up 0 at the same chunk length:
#             the spec kernel then loads exactly the XA stream once, which
#             calibrates bytes per request for its own load pattern
#             (MI355X_MICROARCH.md §HBM: only 16-B/lane streaming reads are
#             calibrated there)
#   summary.json  tools/pmc_summary.py (per-kernel mean durations, counters,
#             HBM traffic per spec launch)
#   usage: tools/profile.sh <tag> [bench args...]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 "$R/bench.py" "$@" > "$OUT/bench.json" 2> "$OUT/trace.log" || {
	echo "trace pass failed rc=$?"; exit 1; }
PM="--steps 5 --warmup 1 --no-cpu --no-verify --no-other"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
    "SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU" \
    "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE" \
    "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run \
      -- python3 "$R/bench.py" "$@" $PM > "$OUT/pmc$i.log" 2>&1 || {
	echo "pmc pass $i ($grp) failed rc=$?"; exit 1; }
done
C=$(python3 -c 'import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["config"]["chunk"])' "$OUT/bench.json")
timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d "$OUT/pmc_w0" -o run \
    -- python3 "$R/bench.py" "$@" $PM --chunk "$C" --warm-blocks 0 > "$OUT/pmc_w0.log" 2>&1 || {
	echo "calibration pass failed rc=$?"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$OUT" --json "$OUT/summary.json" > /dev/null
echo "profile $TAG done"
