set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e21_gpu.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/e21_gpu.log; exit 1; }
tail -1 gpurun_out/e21_gpu.log
L=bjxa_amd/libbjxa.so.0
B="seg=$L:0 noseg=$L:0x40"
for wl in C3 C2; do
timeout -k 10 300 python tools/ab_inproc.py --wl $wl --reps 4 --steps 20 $B > gpurun_out/e21_$wl.log 2>&1
echo == $wl; grep -v amdgpu.ids gpurun_out/e21_$wl.log
done
for mx in W F; do
timeout -k 10 300 python tools/ab_inproc.py --wl C3 --mix $mx --reps 3 --steps 20 $B > gpurun_out/e21_C3$mx.log 2>&1
echo == C3$mx; grep -v amdgpu.ids gpurun_out/e21_C3$mx.log
done
BJXA_LIB_PATH=dbg/times/libbjxa.so.0 timeout -k 10 300 python tools/wave_times.py C3 A > gpurun_out/e21_wt.log 2>&1; tail -2 gpurun_out/e21_wt.log
NOSEG=1 BJXA_LIB_PATH=dbg/times/libbjxa.so.0 timeout -k 10 300 python tools/wave_times.py C3 A > gpurun_out/e21_wtn.log 2>&1; tail -1 gpurun_out/e21_wtn.log
