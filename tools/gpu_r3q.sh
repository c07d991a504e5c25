#!/bin/bash
# bench GPU tests (incl. the other_configs child path), then the driver's
# default bench command, twice
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3/bench_tests.log 2>&1 || { tail -30 gpurun_out/r3/bench_tests.log; exit 1; }
tail -1 gpurun_out/r3/bench_tests.log
for i in 1 2; do
  timeout -k 10 600 python bench.py > gpurun_out/r3/bench_q$i.json 2> gpurun_out/r3/bench_q$i.err || { tail -20 gpurun_out/r3/bench_q$i.err; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(d["value"], d["ms_per_step"], d["ms_per_step_serial"], r["launch_ms"], r["frac"], r["step_frac"], d["bit_exact"]); [print(k, v.get("ms_per_step"), v.get("ms_per_step_serial"), v.get("spec_ms", v.get("kernel_ms")), v.get("frac"), v.get("bit_exact", v.get("byte_exact"))) for k, v in d["other_configs"].items()]' gpurun_out/r3/bench_q$i.json
done
