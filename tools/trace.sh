#!/bin/bash
# Kernel trace + stats of a short bench run: tools/trace.sh <tag> [bench args]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu --no-verify --no-other "$@" > "$OUT/trace.log" 2>&1
echo "trace rc=$?"
