set -o pipefail
mkdir -p gpurun_out
B="base=dbg/base/libbjxa.so.0 mnt=dbg/mnt/libbjxa.so.0 allnt=dbg/allnt/libbjxa.so.0"
for wl in C3 C2 C5g C4; do
timeout -k 10 300 python tools/ab_inproc.py --wl $wl --mix A --reps 4 --steps 20 $B > gpurun_out/aux_$wl.log 2>&1 || { echo "AB $wl failed"; tail -5 gpurun_out/aux_$wl.log; exit 1; }
echo == $wl; grep -v amdgpu.ids gpurun_out/aux_$wl.log
done
