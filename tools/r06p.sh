set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_duplex.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06p_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r06p_tests.log; exit 1; }
BJXA_DUPLEX_OUT2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_duplex.py -x -q --timeout 300 --timeout-method thread >> gpurun_out/r06p_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r06p_tests.log; exit 1; }
grep passed gpurun_out/r06p_tests.log
for ch in 2 1 2; do
timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 12 --alt-env BJXA_DUPLEX_OUT2=0,1 > gpurun_out/r06p.json 2>/dev/null || { echo failed; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['channels'], d['ms_median'])" gpurun_out/r06p.json
done
