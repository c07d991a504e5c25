#!/bin/bash
# issue priority of the second K1 workgroup per CU (variant bits 14-16:
# 1 decode, 2 stores, 4 DMA/LDS), interleaved A/B on C3 and C2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
L=bjxa_amd/libbjxa.so.0
for wl in C3 C2; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl $wl --reps 6 base=$L:0 y1=$L:16384 y2=$L:32768 y3=$L:49152 y7=$L:114688 > gpurun_out/r3/yp_$wl.log 2>&1 || exit $?
  echo $wl; tail -5 gpurun_out/r3/yp_$wl.log
done
