#!/bin/bash
# K2's release before the arrival ticket: __threadfence (base) against a
# release-only agent fence (XA_FIX_REL=1); decode + batch tests on the
# variant, then interleaved A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
L=bjxa_amd/libbjxa.so.0
R=tools/bin/ab/rel.so.0
BJXA_LIB_PATH=$R timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_batch.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/rel_tests.log 2>&1 || { tail -30 gpurun_out/r3/rel_tests.log; exit 1; }
tail -1 gpurun_out/r3/rel_tests.log
for m in A W; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl C3 --mix $m --reps 6 base=$L:0 rel=$R:0 > gpurun_out/r3/rel_c3_$m.log 2>&1 || exit $?
  echo C3 $m; tail -2 gpurun_out/r3/rel_c3_$m.log
done
for wl in C5g C4; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl $wl --reps 5 base=$L:0 rel=$R:0 > gpurun_out/r3/rel_$wl.log 2>&1 || exit $?
  echo $wl; tail -2 gpurun_out/r3/rel_$wl.log
done
