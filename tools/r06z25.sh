# Duplex staging route with 8 staging slots (oldlib/, -DDUPLEX_SLOTS=8)
# against the shipped 4, alternating fresh processes; duplex tests on the
# variant first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
BJXA_LIB_PATH=oldlib/libbjxa.so.0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py > gpurun_out/r06z25_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z25_tests.txt; exit 1; }
tail -1 gpurun_out/r06z25_tests.txt
for i in 1 2 3; do
for ch in 2 1; do
echo "slots8 ch=$ch $(BJXA_LIB_PATH=oldlib/libbjxa.so.0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-120)" || exit 1
echo "slots4 ch=$ch $(timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-120)" || exit 1
done
done
echo "slots8 enc $(BJXA_LIB_PATH=oldlib/libbjxa.so.0 timeout -k 10 200 python tools/host_rate.py --encode --ch 2 --passes 9 | cut -c1-120)" || exit 1
echo "slots4 enc $(timeout -k 10 200 python tools/host_rate.py --encode --ch 2 --passes 9 | cut -c1-120)" || exit 1
