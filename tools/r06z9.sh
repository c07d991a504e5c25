# Duplex decode input: on the decode stream (default) vs every H2D up front
# on an input stream with a stream-write of its count, decodes waiting on
# the count (BJXA_DUPLEX_INQ=val); A/B, tests under val, trace under val
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt9
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_INQ=dec,val || exit 1
done
BJXA_DUPLEX_INQ=val timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py > gpurun_out/r06z9_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z9_tests.txt; exit 1; }
tail -1 gpurun_out/r06z9_tests.txt
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_INQ=val timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt9 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt9/log.txt 2>&1
