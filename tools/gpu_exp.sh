set -o pipefail
mkdir -p gpurun_out
B="cur=bjxa_amd/libbjxa.so.0:0 notail=dbg/notail/libbjxa.so.0:0"
for m in W A; do
timeout -k 10 300 python tools/ab_inproc.py --wl C3 --mix $m --reps 3 --steps 20 $B > gpurun_out/e31.log 2>&1
echo == C3 $m; grep -v amdgpu.ids gpurun_out/e31.log
done
