set -o pipefail
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
B="c64=$L:0 c68=dbg/c68.so:0"
for lay in sep packed gaps sep; do
timeout -k 10 300 python tools/ab_inproc.py --wl C5g --layout $lay --reps 3 --steps 20 $B > gpurun_out/e23.log 2>&1
echo == C5g $lay; grep -v amdgpu.ids gpurun_out/e23.log
done
for lay in sep packed; do
timeout -k 10 300 python tools/ab_inproc.py --wl C4 --layout $lay --reps 3 --steps 20 $B > gpurun_out/e23.log 2>&1
echo == C4 $lay; grep -v amdgpu.ids gpurun_out/e23.log
done
timeout -k 10 300 python tools/ab_inproc.py --wl C5 --layout sep --reps 2 --steps 10 $B > gpurun_out/e23.log 2>&1
echo == C5 sep; grep -v amdgpu.ids gpurun_out/e23.log
