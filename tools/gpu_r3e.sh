#!/bin/bash
# K2 scalar-unit tail repair (SALU clamp, 16-B stores): correctness, then
# mix W / mix A / C4 / C5g A/B against the vector-only K2 (dbg/nosc)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_large.py tests/test_gpu_fuzz.py tests/test_gpu_batch.py > gpurun_out/r3/t3.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3/t3.log
[ $rc -le 1 ] || exit $rc
for m in W A F; do
timeout -k 10 300 python -u tools/ab_inproc.py --wl C3 --mix $m --reps 4 scalar=bjxa_amd/libbjxa.so.0 vector=dbg/nosc/libbjxa.so.0 > gpurun_out/r3/ab2_mix$m.log 2>&1 || exit $?
tail -2 gpurun_out/r3/ab2_mix$m.log
done
for w in C4 C5g; do
timeout -k 10 300 python -u tools/ab_inproc.py --wl $w --reps 3 scalar=bjxa_amd/libbjxa.so.0 vector=dbg/nosc/libbjxa.so.0 > gpurun_out/r3/ab2_$w.log 2>&1 || exit $?
tail -2 gpurun_out/r3/ab2_$w.log
done
