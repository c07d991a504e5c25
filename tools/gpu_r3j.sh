#!/bin/bash
# split-stride batches: GPU tests, then C5g (sep/packed) and C5 A/B of the
# split (variant 0), no split (0x1000) and the full-warm-up split (0x2000)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
L=bjxa_amd/libbjxa.so.0
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/split_tests.log 2>&1 || { tail -30 gpurun_out/r3/split_tests.log; exit 1; }
tail -2 gpurun_out/r3/split_tests.log
for lay in sep packed; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl C5g --layout $lay --reps 4 split=$L:0 nosplit=$L:4096 splitw=$L:8192 > gpurun_out/r3/split_c5g_$lay.log 2>&1 || exit $?
  echo C5g $lay; tail -4 gpurun_out/r3/split_c5g_$lay.log
done
timeout -k 10 300 python -u tools/ab_inproc.py --wl C5 --reps 3 split=$L:0 nosplit=$L:4096 splitw=$L:8192 > gpurun_out/r3/split_c5.log 2>&1 || exit $?
echo C5; tail -4 gpurun_out/r3/split_c5.log
