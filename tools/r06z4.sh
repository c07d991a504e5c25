# Duplex decode: does querying each stream right after enqueueing on it
# (BJXA_DUPLEX_FLUSH=1) let the slabs' input and decodes run beside the
# copy-out?  In-process A/B, then a trace with it on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt4
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_FLUSH=0,1 || exit 1
done
BJXA_DUPLEX_INQ=dec timeout -k 10 200 python tools/host_rate.py --ch 2 --passes 9 --alt-env BJXA_DUPLEX_FLUSH=0,1 || exit 1
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_FLUSH=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt4 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt4/log.txt 2>&1
