# The duplex route as shipped (decode groups to 4, direct encode): all
# duplex and threads tests, a 45 s soak, and host rates for decode and
# encode with the serial routes beside them
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py tests/test_gpu_threads.py tests/test_gpu_encode.py > gpurun_out/r06z18_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z18_tests.txt; exit 1; }
tail -1 gpurun_out/r06z18_tests.txt
timeout -k 10 150 python -u tools/soak_duplex.py --threads 4 --seconds 45 || exit 1
for ch in 2 1; do
BJXA_DUPLEX=0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 || exit 1
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 || exit 1
BJXA_DUPLEX=0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 --encode || exit 1
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 7 --encode || exit 1
done
