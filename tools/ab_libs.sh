#!/bin/bash
# A/B of experimental library builds on the GPU box, interleaved, under
# rocprofv3 --kernel-trace (one box, so the builds are comparable).
#   build:  make -C bjxa_amd/csrc OUT=$PWD/dbg/<v> OBJ=$PWD/dbg/<v>/build EXTRA=-D...
#   run:    VARIANTS="old new" bash tools/ab_libs.sh [C3 C2 ...]
#   read:   python3 tools/trace_kstat.py 'gpurun_out/ab_*/run_results.db'
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
WL=${*:-C3 C2}
export TMPDIR=/tmp
cd /tmp
for r in 1 2; do
for v in $VARIANTS; do
  export BJXA_LIB_PATH=$R/dbg/$v/libbjxa.so.0
  for w in $WL; do
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ab_${v}_${w}${MIX}_$r" -o run \
        -- python3 "$R/bench.py" --no-cpu --no-other --steps 200 --workload $w --mix ${MIX:-A} \
        > "$R/gpurun_out/ab_${v}_${w}${MIX}_$r.log" 2>&1
  done
done
done
