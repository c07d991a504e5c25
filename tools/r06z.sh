# The duplex decode with its PCM written straight into the caller's
# registered buffer (BJXA_DUPLEX_DIRECT=1, the default) against the staging
# copy-out (=0): duplex tests first, then in-process A/B of host-pointer
# bjxa_decode, stereo and mono, a reused and a fresh output buffer
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py > gpurun_out/r06z_duplex_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z_duplex_tests.txt; exit 1; }
tail -1 gpurun_out/r06z_duplex_tests.txt
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_DIRECT=1,0 || exit 1
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 5 --fresh --alt-env BJXA_DUPLEX_DIRECT=1,0 || exit 1
done
BJXA_DUPLEX_TRACE=1 timeout -k 10 100 python tools/host_rate.py --ch 2 --passes 2 2> gpurun_out/r06z_trace.txt || exit 1
