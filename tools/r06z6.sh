# Duplex decode input: copy engine on its own stream (thread), copy engine on
# the decode stream (dec), a copy-in kernel on the decode stream reading the
# registered input (kin); A/B, then the duplex tests and a trace under kin
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt6
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_INQ=thread,dec,kin || exit 1
done
BJXA_DUPLEX_INQ=kin timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py > gpurun_out/r06z6_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z6_tests.txt; exit 1; }
tail -1 gpurun_out/r06z6_tests.txt
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_INQ=kin timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt6 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt6/log.txt 2>&1
