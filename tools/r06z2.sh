# The duplex decode's input H2D on its own stream (input thread, BJXA_DUPLEX_INQ
# unset) vs on the decode stream (=dec): in-process A/B, stereo and mono,
# then a kernel + copy trace of the =dec route
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06zt2
for ch in 2 1; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 --alt-env BJXA_DUPLEX_INQ=thread,dec || exit 1
done
BJXA_DUPLEX_INQ=dec BJXA_DUPLEX_TRACE=1 timeout -k 10 100 python tools/host_rate.py --ch 2 --passes 2 2> gpurun_out/r06z2_trace.txt || exit 1
cd /tmp && export TMPDIR=/tmp
BJXA_DUPLEX_INQ=dec timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06zt2 -o run -- python3 $GRAFT_REPO_ROOT/tools/host_rate.py --ch 2 --passes 2 > $GRAFT_REPO_ROOT/gpurun_out/r06zt2/log.txt 2>&1
