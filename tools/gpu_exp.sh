set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e14_gpu.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/e14_gpu.log; exit 1; }
tail -2 gpurun_out/e14_gpu.log
export TMPDIR=/tmp
L=$R/bjxa_amd/libbjxa.so.0
for wl in C5g C4; do for mx in Z A W; do
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/e14_tr$wl$mx -o run -- python3 $R/tools/ab_inproc.py --wl $wl --mix $mx --reps 2 --steps 20 d=$L:0 > $R/gpurun_out/e14_tr$wl$mx.log 2>&1 )
echo == $wl $mx; grep -h "xa_decode" gpurun_out/e14_tr$wl$mx/*kernel_stats.csv | cut -d, -f1-4
done; done
