# Duplex decode, every slab in flight on the direct route: slabs per decode
# launch (BJXA_DUPLEX_GROUP = 1 / 2 / 4 / 8);
# slab 0 alone, then 2, then up to the cap): A/B, the duplex tests under 4,
# and a trace under 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt12
BJXA_DUPLEX_GROUP=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py > gpurun_out/r06z12_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z12_tests.txt; exit 1; }
tail -1 gpurun_out/r06z12_tests.txt
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_GROUP=1,2,4,8 || exit 1
done
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_GROUP=8 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt12 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt12/log.txt 2>&1
