#!/bin/bash
# four-group K1 (variant 0x10): parity tests, then interleaved A/B on C3/C2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
L=bjxa_amd/libbjxa.so.0
timeout -k 10 400 python -u -m pytest tests/test_gpu_longrun.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/lr_tests.log 2>&1 || { tail -30 gpurun_out/r3/lr_tests.log; exit 1; }
tail -1 gpurun_out/r3/lr_tests.log
for wl in C3 C2; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl $wl --reps 5 base=$L:0 lr=$L:16 > gpurun_out/r3/lr_$wl.log 2>&1 || exit $?
  echo $wl; tail -2 gpurun_out/r3/lr_$wl.log
done
