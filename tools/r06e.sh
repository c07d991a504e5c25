# the duplex host-pointer route: parity, then bjxa_decode() timings with it
# on and off (BJXA_DUPLEX=0), alternating processes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_duplex.py tests/test_gpu_api.py tests/test_gpu_threads.py tests/test_gpu_small.py tests/test_gpu_decode.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06e_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r06e_tests.log; exit 1; }
tail -3 gpurun_out/r06e_tests.log
for rep in 1 2; do
for d in 1 0; do
for ch in 2 1; do
BJXA_DUPLEX=$d timeout -k 10 120 python tools/host_rate.py --ch $ch --passes 7 > gpurun_out/r06e_host_d${d}_ch${ch}_$rep.json 2>/dev/null || { echo "host_rate failed"; exit 1; }
echo "duplex=$d $(cat gpurun_out/r06e_host_d${d}_ch${ch}_$rep.json)"
done
done
done
