set -o pipefail
mkdir -p gpurun_out
R=$PWD
L=bjxa_amd/libbjxa.so.0
B="base=dbg/base.so:0 new=$L:0 rel=dbg/rel.so:0"
for mx in A W F; do
timeout -k 10 300 python tools/ab_inproc.py --wl C3 --mix $mx --reps 4 --steps 20 $B > gpurun_out/e11_C3$mx.log 2>&1
echo == C3$mx; grep -v amdgpu.ids gpurun_out/e11_C3$mx.log
done
export TMPDIR=/tmp
for mx in Z A W; do
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/e11_tr$mx -o run -- python3 $R/bench.py --mix $mx --no-other --no-cpu --no-verify --steps 50 > $R/gpurun_out/e11_tr$mx.log 2>&1 )
echo == trace $mx; grep -h "xa_decode" gpurun_out/e11_tr$mx/*kernel_stats.csv | cut -d, -f1-4
done
