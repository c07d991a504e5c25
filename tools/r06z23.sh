# The duplex route with every kernel enqueued up front and only the copy-outs
# gated by the staging slots: duplex tests, threads tests, host rates (staging,
# direct, serial), a 30 s soak
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py tests/test_gpu_threads.py > gpurun_out/r06z23_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z23_tests.txt; exit 1; }
tail -1 gpurun_out/r06z23_tests.txt
for ch in 2 1; do
echo "serial ch=$ch $(BJXA_DUPLEX=0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 | cut -c1-120)" || exit 1
echo "staging ch=$ch $(timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-120)" || exit 1
echo "direct ch=$ch $(BJXA_DUPLEX_DIRECT=1 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-120)" || exit 1
echo "staging enc ch=$ch $(timeout -k 10 200 python tools/host_rate.py --encode --ch $ch --passes 9 | cut -c1-120)" || exit 1
done
timeout -k 10 100 python -u tools/soak_duplex.py --threads 4 --seconds 30 || exit 1
