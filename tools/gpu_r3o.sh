#!/bin/bash
# round-3 profile set: suite, smoke, default bench line, C3 trace + counters
# (tools/gpu_round.sh), then kernel traces of C5 and its per-GPU shares
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r03c || exit 1
for s in "c5 --workload C5 --steps 20" "c5n2 --workload C5 --streams 512 --steps 20" \
         "c5n4 --workload C5 --streams 256 --steps 30" "c5n8 --workload C5 --streams 128 --steps 50"; do
  set -- $s
  T=r03c_$1; shift
  bash tools/trace.sh $T "$@" || exit 1
  python3 tools/pmc_summary.py gpurun_out/prof_$T --json gpurun_out/prof_$T/summary.json > /dev/null || exit 1
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k: v for k, v in d["kernel_us_alone"].items() if "xa_" in k})' gpurun_out/prof_$T/summary.json
done
