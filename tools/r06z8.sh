# The reworked duplex route (input on the decode stream, PCM straight into
# a resident registered caller buffer): duplex + decode + threads tests,
# then host-pointer rates: decode stereo/mono with BJXA_DUPLEX_DIRECT=1,0
# (reused and fresh output), the serial route (BJXA_DUPLEX=0 in a child),
# and the encode route
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py tests/test_gpu_threads.py tests/test_gpu_api.py > gpurun_out/r06z8_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z8_tests.txt; exit 1; }
tail -1 gpurun_out/r06z8_tests.txt
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_DIRECT=1,0 || exit 1
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 5 --fresh --alt-env BJXA_DUPLEX_DIRECT=1,0 || exit 1
BJXA_DUPLEX=0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 || exit 1
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 || exit 1
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 --encode || exit 1
done
BJXA_DUPLEX_TRACE=1 timeout -k 10 100 python tools/host_rate.py --ch 2 --passes 2 2> gpurun_out/r06z8_trace.txt || exit 1
