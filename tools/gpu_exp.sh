set -o pipefail
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
B="off=$L:0xf00 g1=$L:0x100 g2=$L:0x200 g4=$L:0x400 g8=$L:0x800"
for wl in C3 C2 C5g C4; do
timeout -k 10 300 python tools/ab_inproc.py --wl $wl --reps 6 --steps 20 $B > gpurun_out/ab4_$wl.log 2>&1
echo == $wl; grep -v amdgpu.ids gpurun_out/ab4_$wl.log
done
timeout -k 10 300 python tools/ab_inproc.py --wl C5 --reps 4 --steps 10 $B > gpurun_out/ab4_C5.log 2>&1
echo == C5; grep -v amdgpu.ids gpurun_out/ab4_C5.log
