set -o pipefail
mkdir -p gpurun_out
T=${1:-r2f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${T}_gpu.log; exit 1; }
tail -2 gpurun_out/${T}_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH FAILED; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(d["value"], d["ms_per_step"], d["ms_per_step_serial"], r["launch_ms"], r["frac"], r["step_frac"], d["bit_exact"]); [print(k, v.get("ms_per_step"), v.get("ms_per_step_serial"), v.get("spec_ms", v.get("kernel_ms")), v.get("frac")) for k, v in d["other_configs"].items()]' gpurun_out/${T}_bench.json
[ "${2:-prof}" = noprof ] && exit 0
bash tools/profile.sh $T || exit 1
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["kernel_us"], d["kernel_us_alone"], d.get("traffic"))' gpurun_out/prof_$T/summary.json
