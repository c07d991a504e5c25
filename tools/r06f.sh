set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for cfg in "1 0" "2 0" "4 0" "16 0" "1 1" "4 1"; do
set -- $cfg
if [ "$2" = 1 ]; then export BJXA_DUPLEX_REG=1; else unset BJXA_DUPLEX_REG; fi
BJXA_DUPLEX_IN=$1 timeout -k 10 120 python tools/host_rate.py --ch 2 --passes 5 > gpurun_out/r06f_host_$1_$2.json 2>/dev/null || { echo failed; exit 1; }
echo "in=$1 reg=$2 $(cat gpurun_out/r06f_host_$1_$2.json)"
done
BJXA_DUPLEX_IN=4 BJXA_DUPLEX_TRACE=1 timeout -k 10 120 python tools/host_rate.py --ch 2 --passes 1 > /dev/null 2> gpurun_out/r06f_trace4.txt || exit 1
BJXA_DUPLEX_REG=1 BJXA_DUPLEX_TRACE=1 timeout -k 10 120 python tools/host_rate.py --ch 2 --passes 1 > /dev/null 2> gpurun_out/r06f_trace_reg.txt || exit 1
grep -v amdgpu.ids gpurun_out/r06f_trace4.txt | tail -18; grep -v amdgpu.ids gpurun_out/r06f_trace_reg.txt | tail -19
