# full GPU suite with the duplex route in, then the host-pointer call both ways
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06h_gpu.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r06h_gpu.log; exit 1; }
tail -2 gpurun_out/r06h_gpu.log
for rep in 1 2 3; do
for d in 1 0; do
for ch in 2 1; do
BJXA_DUPLEX=$d timeout -k 10 120 python tools/host_rate.py --ch $ch --passes 7 > gpurun_out/r06h_host_d${d}_ch${ch}_$rep.json 2>/dev/null || { echo "host_rate failed"; exit 1; }
echo "duplex=$d ch=$ch $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms'], d['bit_exact'])" gpurun_out/r06h_host_d${d}_ch${ch}_$rep.json)"
done
done
done
