set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/swz_gpu.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/swz_gpu.log; exit 1; }
tail -2 gpurun_out/swz_gpu.log
B="base=dbg/base/libbjxa.so.0 swz=bjxa_amd/libbjxa.so.0"
for wl in C3 C2 C4 C5g; do
timeout -k 10 300 python tools/ab_inproc.py --wl $wl --mix A --reps 4 --steps 20 $B > gpurun_out/swz_$wl.log 2>&1 || { echo "AB $wl failed"; tail -5 gpurun_out/swz_$wl.log; exit 1; }
echo == $wl; grep -v amdgpu.ids gpurun_out/swz_$wl.log
done
