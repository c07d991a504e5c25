#!/bin/bash
# repair-chain latency form (XA_FIX_LAT): decode/batch GPU tests with it,
# then interleaved A/B against a build without it (tools/bin/ab/nolat.so.0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
L=bjxa_amd/libbjxa.so.0
N=tools/bin/ab/nolat.so.0
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_batch.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/lat_tests.log 2>&1 || { tail -30 gpurun_out/r3/lat_tests.log; exit 1; }
tail -2 gpurun_out/r3/lat_tests.log
for m in A W; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl C3 --mix $m --reps 5 lat=$L:0 nolat=$N:0 > gpurun_out/r3/lat_c3_$m.log 2>&1 || exit $?
  echo C3 mix $m; tail -2 gpurun_out/r3/lat_c3_$m.log
done
timeout -k 10 300 python -u tools/ab_inproc.py --wl C5g --reps 4 lat=$L:0 nolat=$N:0 > gpurun_out/r3/lat_c5g.log 2>&1 || exit $?
echo C5g; tail -2 gpurun_out/r3/lat_c5g.log
