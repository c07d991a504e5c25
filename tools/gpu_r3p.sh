#!/bin/bash
# batch K2 shape: 256 x 4-wave workgroups (base), up to 1024 x 4 (wg1k),
# 256 x 8 (wpb8); batch tests on both variants, then interleaved A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
L=bjxa_amd/libbjxa.so.0
for v in wg1k wpb8; do
  BJXA_LIB_PATH=tools/bin/ab/$v.so.0 timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/fixb_tests_$v.log 2>&1 || { tail -20 gpurun_out/r3/fixb_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r3/fixb_tests_$v.log
done
for wl in C5g C5 C4; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl $wl --reps 5 base=$L:0 wg1k=tools/bin/ab/wg1k.so.0:0 wpb8=tools/bin/ab/wpb8.so.0:0 > gpurun_out/r3/fixb_$wl.log 2>&1 || exit $?
  echo $wl; tail -3 gpurun_out/r3/fixb_$wl.log
done
