# Duplex encode writing its XA straight into the registered caller buffer
# (direct, every slab in flight) with encode groups BJXA_DUPLEX_EGROUP =
# 1 / 4 / 8 / 16, and the staging route (BJXA_DUPLEX_DIRECT=0): encode tests
# under direct + 8 and under staging, in-process A/B, a trace under 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt17
BJXA_DUPLEX_EGROUP=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py -k encode > gpurun_out/r06z17_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z17_tests.txt; exit 1; }
BJXA_DUPLEX_DIRECT=0 BJXA_DUPLEX_EGROUP=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py -k encode >> gpurun_out/r06z17_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z17_tests.txt; exit 1; }
grep passed gpurun_out/r06z17_tests.txt
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --encode --ch $ch --passes 9 --alt-env BJXA_DUPLEX_EGROUP=1,4,8,16 || exit 1
done
BJXA_DUPLEX_DIRECT=0 timeout -k 10 200 python tools/host_rate.py --encode --ch 2 --passes 9 --alt-env BJXA_DUPLEX_EGROUP=1,2 || exit 1
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_EGROUP=8 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt17 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --encode --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt17/log.txt 2>&1
