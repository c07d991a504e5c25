# Duplex encode: slabs per encode launch (BJXA_DUPLEX_EGROUP = 1 / 2 / 4,
# groups growing 1, 2, 3, 4 within the 4 staging slots): encode tests under
# 4, in-process A/B, a trace under 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt16
BJXA_DUPLEX_EGROUP=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py -k encode > gpurun_out/r06z16_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z16_tests.txt; exit 1; }
tail -1 gpurun_out/r06z16_tests.txt
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --encode --ch $ch --passes 9 --alt-env BJXA_DUPLEX_EGROUP=1,2,4 || exit 1
done
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_EGROUP=4 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt16 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --encode --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt16/log.txt 2>&1
