set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
BJXA_DUPLEX_KIN=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_duplex.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06i_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r06i_tests.log; exit 1; }
tail -1 gpurun_out/r06i_tests.log
for rep in 1 2; do
for kin in 1 0; do
if [ $kin = 1 ]; then export BJXA_DUPLEX_KIN=1; else unset BJXA_DUPLEX_KIN; fi
for mode in "" "--encode"; do
timeout -k 10 120 python tools/host_rate.py $mode --ch 2 --passes 7 > gpurun_out/r06i.json 2>/dev/null || { echo "host_rate failed"; exit 1; }
echo "kin=$kin $mode $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms'], d.get('bit_exact', d.get('byte_exact')))" gpurun_out/r06i.json)"
done
done
done
export BJXA_DUPLEX_KIN=1
BJXA_DUPLEX_TRACE=1 timeout -k 10 120 python tools/host_rate.py --ch 2 --passes 1 > /dev/null 2> gpurun_out/r06i_trace.txt || exit 1
grep -v amdgpu.ids gpurun_out/r06i_trace.txt | tail -18
