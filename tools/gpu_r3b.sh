#!/bin/bash
# Region kernel vs lane-strided K1 on C3: instruction-cache and issue counters
# (one counter group per rocprofv3 pass).
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3/pmc_b
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
AB="$R/tools/ab_inproc.py --wl C3 --reps 1 --steps 5 region=$R/bjxa_amd/libbjxa.so.0:128 strided=$R/bjxa_amd/libbjxa.so.0:0"
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
    "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $AB > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo done
