#!/bin/bash
# K2 scalar-unit tail repair: correctness, then mix W / mix A A/B against the
# vector-only K2 (dbg/nosc); K1 workgroup shape x chunk plan A/B; timelines.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_large.py tests/test_gpu_fuzz.py tests/test_gpu_batch.py tests/test_gpu_dist.py > gpurun_out/r3/t2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3/t2.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_inproc.py --wl C3 --mix W --reps 4 scalar=bjxa_amd/libbjxa.so.0 vector=dbg/nosc/libbjxa.so.0 > gpurun_out/r3/ab_mixw.log 2>&1 || exit $?
tail -3 gpurun_out/r3/ab_mixw.log
timeout -k 10 300 python -u tools/ab_inproc.py --wl C3 --mix A --reps 4 scalar=bjxa_amd/libbjxa.so.0 vector=dbg/nosc/libbjxa.so.0 > gpurun_out/r3/ab_mixa.log 2>&1 || exit $?
tail -3 gpurun_out/r3/ab_mixa.log
timeout -k 10 400 python -u tools/ab_inproc.py --wl C3 --reps 4 base=bjxa_amd/libbjxa.so.0:0 bal=bjxa_amd/libbjxa.so.0:32 w8=dbg/wpb8/libbjxa.so.0:0 w8bal=dbg/wpb8/libbjxa.so.0:32 > gpurun_out/r3/ab_shape.log 2>&1 || exit $?
tail -5 gpurun_out/r3/ab_shape.log
BJXA_LIB_PATH=dbg/wpb8t/libbjxa.so.0 timeout -k 10 120 python -u tools/wave_times.py C3 A 32 _w8bal > gpurun_out/r3/wt_w8bal.log 2>&1 || exit $?
BJXA_LIB_PATH=dbg/times/libbjxa.so.0 timeout -k 10 120 python -u tools/wave_times.py C3 A 32 _bal > gpurun_out/r3/wt_bal.log 2>&1 || exit $?
tail -1 gpurun_out/r3/wt_w8bal.log; tail -1 gpurun_out/r3/wt_bal.log
