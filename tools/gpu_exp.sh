set -o pipefail
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
for wl in C3 C2; do
timeout -k 10 300 python tools/ab_inproc.py --wl $wl --mix A --reps 3 --steps 20 auto=$L:0 bal=$L:32 > gpurun_out/e33.log 2>&1 || exit 1
echo == $wl A; grep -v amdgpu.ids gpurun_out/e33.log
done
