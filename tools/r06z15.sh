# Duplex decode with one workspace per group shape (this tree) against the
# previous build (oldlib/, one shared workspace): duplex tests, then host
# rates in alternating fresh processes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py > gpurun_out/r06z15_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z15_tests.txt; exit 1; }
tail -1 gpurun_out/r06z15_tests.txt
for i in 1 2 3; do
for ch in 2 1; do
echo "old ch=$ch $(BJXA_LIB_PATH=oldlib/libbjxa.so.0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-160)" || exit 1
echo "new ch=$ch $(timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-160)" || exit 1
done
done
BJXA_DUPLEX_TRACE=1 timeout -k 10 100 python tools/host_rate.py --ch 2 --passes 2 2> gpurun_out/r06z15_trace.txt || exit 1
