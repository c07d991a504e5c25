# The duplex route as shipped (decode groups capped at 4, every slab in
# flight on the direct route): duplex tests, a 45 s 4-thread soak, and the
# host-pointer rates (serial route in a child with BJXA_DUPLEX=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py tests/test_gpu_threads.py > gpurun_out/r06z14_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z14_tests.txt; exit 1; }
tail -1 gpurun_out/r06z14_tests.txt
timeout -k 10 150 python -u tools/soak_duplex.py --threads 4 --seconds 45 || exit 1
for ch in 2 1; do
BJXA_DUPLEX=0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 || exit 1
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 || exit 1
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 5 --fresh --alt-env BJXA_DUPLEX_DIRECT=1,0 || exit 1
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 --encode || exit 1
done
BJXA_DUPLEX_TRACE=1 timeout -k 10 100 python tools/host_rate.py --ch 2 --passes 2 2> gpurun_out/r06z14_trace.txt || exit 1
