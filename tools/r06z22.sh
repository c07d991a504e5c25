# The duplex route with the direct output opt-in: duplex tests, then host
# rates on the default (staging) route and with BJXA_DUPLEX_DIRECT=1, and the
# serial route, in fresh processes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py > gpurun_out/r06z22_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z22_tests.txt; exit 1; }
tail -1 gpurun_out/r06z22_tests.txt
for ch in 2 1; do
echo "serial ch=$ch $(BJXA_DUPLEX=0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 | cut -c1-120)" || exit 1
echo "staging ch=$ch $(timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-120)" || exit 1
echo "direct ch=$ch $(BJXA_DUPLEX_DIRECT=1 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-120)" || exit 1
echo "staging enc ch=$ch $(timeout -k 10 200 python tools/host_rate.py --encode --ch $ch --passes 9 | cut -c1-120)" || exit 1
done
