# Duplex decode: the input H2D on a CU-masked stream of its own
# (BJXA_DUPLEX_INQ=masked) vs the plain input stream; A/B then a trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt5
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_INQ=thread,masked,dec || exit 1
done
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_INQ=masked timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt5 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt5/log.txt 2>&1
