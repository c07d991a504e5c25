set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py -x -q --timeout 280 --timeout-method thread > gpurun_out/p2_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/p2_tests.log; exit 1; }
tail -2 gpurun_out/p2_tests.log
for d in 1 2; do
bash tools/trace.sh pipe$d --pipeline $d --steps 30 || exit 1
python3 tools/trace_overlap.py gpurun_out/prof_pipe$d
done
