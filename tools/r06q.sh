set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
BJXA_DUPLEX_GROUP=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_duplex.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06q_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r06q_tests.log; exit 1; }
grep passed gpurun_out/r06q_tests.log
for ch in 2 1 2; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 12 --alt-env BJXA_DUPLEX_GROUP=1,4,8 > gpurun_out/r06q.json 2>/dev/null || { echo failed; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['channels'], d['ms_median'])" gpurun_out/r06q.json
done
BJXA_DUPLEX_GROUP=4 BJXA_DUPLEX_TRACE=1 timeout -k 10 120 python tools/host_rate.py --ch 2 --passes 1 > /dev/null 2> gpurun_out/r06q_trace.txt || exit 1
grep -v amdgpu.ids gpurun_out/r06q_trace.txt | tail -18
