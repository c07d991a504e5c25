#!/bin/bash
# The driver's default bench line, then the same with BJXA_CPU_THREADS=16 off
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u bench.py > gpurun_out/r3/bench_default.json 2> gpurun_out/r3/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r3/bench_default.json
