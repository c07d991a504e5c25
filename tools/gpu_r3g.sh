#!/bin/bash
# Two-phase plan (persistent K1, run-time tail tasks): tests, then A/B on
# C3 and C2 against the current plan; region-kernel tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_large.py tests/test_gpu_region.py tests/test_gpu_decode.py > gpurun_out/r3/t4.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r3/t4.log
[ $rc -le 1 ] || exit $rc
L=bjxa_amd/libbjxa.so.0
timeout -k 10 400 python -u tools/ab_inproc.py --wl C3 --reps 4 base=$L:0 tp=$L:4096 tp28=$L:4096:28 tp36=$L:4096:36 > gpurun_out/r3/ab_tp_c3.log 2>&1 || exit $?
tail -4 gpurun_out/r3/ab_tp_c3.log
timeout -k 10 400 python -u tools/ab_inproc.py --wl C3 --mix W --reps 3 base=$L:0 tp=$L:4096 > gpurun_out/r3/ab_tp_c3w.log 2>&1 || exit $?
tail -2 gpurun_out/r3/ab_tp_c3w.log
timeout -k 10 400 python -u tools/ab_inproc.py --wl C2 --reps 4 base=$L:0 tp=$L:4096 tp56=$L:4096:56 > gpurun_out/r3/ab_tp_c2.log 2>&1 || exit $?
tail -3 gpurun_out/r3/ab_tp_c2.log
