set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_gpu3.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r2_gpu1.log; exit 1; }
tail -3 gpurun_out/r2_gpu3.log
gcc -O2 -Iinclude -o gpurun_out/call_latency tools/call_latency.c bjxa_amd/libbjxa.so.0 -Wl,-rpath,$PWD/bjxa_amd
timeout -k 10 300 gpurun_out/call_latency > gpurun_out/r2_call_latency3.json
timeout -k 10 400 python bench.py > gpurun_out/r2_bench3.log 2> gpurun_out/r2_bench3.err
tail -c 600 gpurun_out/r2_bench3.log
