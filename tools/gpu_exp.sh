set -o pipefail
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
timeout -k 10 300 python tools/ab_inproc.py --wl C5g --mix A --reps 4 --steps 20 d=$L c192=$L:0:192 c256=$L:0:256 w4=$L:0:0:4 > gpurun_out/c5g_tune.log 2>&1 || { echo "AB failed"; tail -5 gpurun_out/c5g_tune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c5g_tune.log
timeout -k 10 300 python tools/ab_inproc.py --wl C4 --mix A --reps 3 --steps 20 d=$L c256=$L:0:256 c320=$L:0:320 > gpurun_out/c4_tune.log 2>&1 || { echo "AB failed"; tail -5 gpurun_out/c4_tune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c4_tune.log
