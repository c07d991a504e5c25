#!/bin/bash
# GPU suite, then the per-wave K1 timeline (diagnostic build in dbg/times)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -4 gpurun_out/r3/gpu_suite.log
[ $rc -le 1 ] || exit $rc
BJXA_LIB_PATH=dbg/times/libbjxa.so.0 timeout -k 10 120 python -u tools/wave_times.py C3 A > gpurun_out/r3/wt_c3.log 2>&1
echo "wt rc=$?"; tail -2 gpurun_out/r3/wt_c3.log
