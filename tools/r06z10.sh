# Duplex decode writing its PCM straight into the registered caller buffer
# from the decode kernel (BJXA_DUPLEX_ZC=1, experiment: no copy-out) vs the
# copy-out route; A/B, then a trace under ZC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt10
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_ZC=0,1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_ZC=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt10 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt10/log.txt 2>&1
