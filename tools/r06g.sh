set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export BJXA_DUPLEX_REG=1
for rep in 1 2; do
for nc in 0 1; do
if [ $nc = 1 ]; then export BJXA_DUPLEX_NOCOPY=1; else unset BJXA_DUPLEX_NOCOPY; fi
for t in 16 8; do
BJXA_THREADS=$t timeout -k 10 120 python tools/host_rate.py --ch 2 --passes 5 > gpurun_out/r06g_n$nc.json 2>/dev/null || { echo failed; exit 1; }
echo "nocopy=$nc threads=$t $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms'], d['bit_exact'])" gpurun_out/r06g_n$nc.json)"
done
done
done
unset BJXA_DUPLEX_NOCOPY
BJXA_DUPLEX_NOCOPY=1 BJXA_DUPLEX_TRACE=1 timeout -k 10 120 python tools/host_rate.py --ch 2 --passes 1 > /dev/null 2> gpurun_out/r06g_trace_nc.txt || exit 1
grep -v amdgpu.ids gpurun_out/r06g_trace_nc.txt | tail -18
