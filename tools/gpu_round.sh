set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2f_gpu.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r2f_gpu.log; exit 1; }
tail -3 gpurun_out/r2f_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2f_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/r2f_smoke.log; exit 1; }
tail -1 gpurun_out/r2f_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r2f_bench.json 2> gpurun_out/r2f_bench.err || { echo BENCH FAILED; tail -20 gpurun_out/r2f_bench.err; exit 1; }
cat gpurun_out/r2f_bench.json
