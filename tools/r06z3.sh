# The duplex decode's input H2D: own stream (thread), the codec's main
# stream (main), the decode stream (dec); in-process A/B, then a trace of main
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt3
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_INQ=thread,main,dec || exit 1
done
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_INQ=main timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt3 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt3/log.txt 2>&1
