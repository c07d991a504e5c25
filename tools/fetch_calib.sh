#!/bin/bash
# Calibrate FETCH_SIZE for the decode's own load pattern (GPU box).
# MI355X_MICROARCH.md §HBM: only 16-B/lane streaming reads are calibrated;
# the spec kernel stages 4-B/lane LDS-DMA.  With warm-up W the kernel loads
# exactly (C + W) / C x the XA stream, so TCC_EA0_RDREQ at several W gives
# bytes per request by regression on a known byte count.
#   usage: tools/fetch_calib.sh <tag> [bench args...]
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/calib_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for W in 0 8 16; do
  timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv \
      -d "$OUT/w$W" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-verify --no-other \
      --chunk 40 --warm-blocks $W "$@" > "$OUT/w$W.log" 2>&1
done
echo "calib $TAG done"
