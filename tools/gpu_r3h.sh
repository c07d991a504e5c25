#!/bin/bash
# Store grouping A/B (variant 0x10: each store instruction covers the lines of
# chunks 8 apart instead of 8 consecutive chunks)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
L=bjxa_amd/libbjxa.so.0
for w in C5g C3 C4 C2; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl $w --reps 4 base=$L:0 il=$L:16 > gpurun_out/r3/ab_il_$w.log 2>&1 || exit $?
  echo $w; tail -2 gpurun_out/r3/ab_il_$w.log
done
timeout -k 10 300 python -u tools/ab_inproc.py --wl C5g --layout packed --reps 3 base=$L:0 il=$L:16 > gpurun_out/r3/ab_il_C5g_packed.log 2>&1 || exit $?
echo C5g packed; tail -2 gpurun_out/r3/ab_il_C5g_packed.log
timeout -k 10 300 python -u tools/ab_inproc.py --wl C5 --reps 2 base=$L:0 il=$L:16 > gpurun_out/r3/ab_il_C5.log 2>&1 || exit $?
echo C5; tail -2 gpurun_out/r3/ab_il_C5.log
