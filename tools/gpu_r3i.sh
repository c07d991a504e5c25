#!/bin/bash
# C5g under stream placements: separate allocations, back to back, random
# gaps of 0-64 KiB / 0-2 MiB, a structured skew
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
L=bjxa_amd/libbjxa.so.0
for lay in sep packed gaps gaps2m skew sep; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl C5g --layout $lay --reps 3 base=$L:0 > gpurun_out/r3/lay_$lay.log 2>&1 || exit $?
  echo $lay; tail -1 gpurun_out/r3/lay_$lay.log
done
