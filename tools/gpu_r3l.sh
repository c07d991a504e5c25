#!/bin/bash
# full GPU suite on the committed build, then K2's grid (chunk boundaries
# per thread XA_FIX_CPT 2 = default, 4, 8: 245 / 123 / 62 workgroups on C3)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
L=bjxa_amd/libbjxa.so.0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3/suite_l.log 2>&1 || { tail -30 gpurun_out/r3/suite_l.log; exit 1; }
tail -2 gpurun_out/r3/suite_l.log
for m in Z A W; do
  timeout -k 10 300 python -u tools/ab_inproc.py --wl C3 --mix $m --reps 5 cpt2=$L:0 cpt4=tools/bin/ab/cpt4.so.0:0 cpt8=tools/bin/ab/cpt8.so.0:0 > gpurun_out/r3/cpt_c3_$m.log 2>&1 || exit $?
  echo C3 mix $m; tail -3 gpurun_out/r3/cpt_c3_$m.log
done
timeout -k 10 300 python -u tools/ab_inproc.py --wl C2 --reps 5 cpt2=$L:0 cpt4=tools/bin/ab/cpt4.so.0:0 cpt8=tools/bin/ab/cpt8.so.0:0 > gpurun_out/r3/cpt_c2.log 2>&1 || exit $?
echo C2; tail -3 gpurun_out/r3/cpt_c2.log
