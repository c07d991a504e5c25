set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./dbg/repair_probe_old > gpurun_out/e32_rep_old.log 2>&1 || exit 1
timeout -k 10 120 ./dbg/repair_probe > gpurun_out/e32_rep_lat.log 2>&1 || exit 1
echo == probe old; head -10 gpurun_out/e32_rep_old.log | grep '"buf": 1'
echo == probe lat; head -10 gpurun_out/e32_rep_lat.log | grep '"buf": 1'
B="base=dbg/base/libbjxa.so.0:0 lat=bjxa_amd/libbjxa.so.0:0"
for m in W A; do
timeout -k 10 300 python tools/ab_inproc.py --wl C3 --mix $m --reps 3 --steps 20 $B > gpurun_out/e32.log 2>&1 || exit 1
echo == C3 $m; grep -v amdgpu.ids gpurun_out/e32.log
done
for m in A W; do
timeout -k 10 300 python tools/ab_inproc.py --wl C4 --mix $m --reps 3 --steps 20 $B > gpurun_out/e32.log 2>&1 || exit 1
echo == C4 $m; grep -v amdgpu.ids gpurun_out/e32.log
done
timeout -k 10 300 python tools/ab_inproc.py --wl C2 --mix W --reps 3 --steps 20 $B > gpurun_out/e32.log 2>&1 || exit 1
echo == C2 W; grep -v amdgpu.ids gpurun_out/e32.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e32_gpu.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/e32_gpu.log; exit 1; }
tail -2 gpurun_out/e32_gpu.log
