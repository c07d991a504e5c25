# Duplex route with its events kept across calls (this tree) against
# events made per call (oldlib/, the previous build): duplex tests, then
# alternating fresh processes, decode and encode
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py tests/test_gpu_threads.py > gpurun_out/r06z20_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z20_tests.txt; exit 1; }
tail -1 gpurun_out/r06z20_tests.txt
for i in 1 2 3; do
for ch in 2 1; do
echo "percall ch=$ch $(BJXA_LIB_PATH=oldlib/libbjxa.so.0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-130)" || exit 1
echo "pooled  ch=$ch $(timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-130)" || exit 1
done
echo "percall enc $(BJXA_LIB_PATH=oldlib/libbjxa.so.0 timeout -k 10 200 python tools/host_rate.py --encode --ch 2 --passes 9 | cut -c1-130)" || exit 1
echo "pooled  enc $(timeout -k 10 200 python tools/host_rate.py --encode --ch 2 --passes 9 | cut -c1-130)" || exit 1
done
