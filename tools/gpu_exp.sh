set -o pipefail
mkdir -p gpurun_out
B="wpb4=bjxa_amd/libbjxa.so.0:0 wpb8=dbg/wpb8/libbjxa.so.0:0"
for wl in C3 C2 C4 C5g; do
timeout -k 10 300 python tools/ab_inproc.py --wl $wl --mix A --reps 3 --steps 20 $B > gpurun_out/e34.log 2>&1 || exit 1
echo == $wl A; grep -v amdgpu.ids gpurun_out/e34.log
done
