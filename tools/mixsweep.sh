#!/bin/bash
# GPU tests, then the default decode step on C3 for profile mixes A, W, F
# (GPU box).  usage: tools/mixsweep.sh <tag> [sweep args...]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd "$R"
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc = 0 ] || exit 1
for M in A W F; do
  timeout -k 10 200 python tools/sweep.py --mix $M --steps 30 "$@" 2>&1 | grep -v amdgpu.ids || exit 1
done
