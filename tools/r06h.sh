# duplex route: decode + encode parity, then host-pointer timings both ways
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_duplex.py tests/test_gpu_encode.py tests/test_gpu_api.py tests/test_gpu_threads.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06h_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r06h_tests.log; exit 1; }
tail -2 gpurun_out/r06h_tests.log
for rep in 1 2 3; do
for d in 1 0; do
for ch in 2 1; do
BJXA_DUPLEX=$d timeout -k 10 120 python tools/host_rate.py --encode --ch $ch --passes 7 > gpurun_out/r06h_enc_d${d}_ch${ch}_$rep.json 2>/dev/null || { echo "host_rate failed"; exit 1; }
echo "encode duplex=$d ch=$ch $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms'], d['byte_exact'])" gpurun_out/r06h_enc_d${d}_ch${ch}_$rep.json)"
done
done
done
BJXA_DUPLEX_TRACE=1 timeout -k 10 120 python tools/host_rate.py --encode --ch 2 --passes 1 > /dev/null 2> gpurun_out/r06h_enc_trace.txt || exit 1
grep -v amdgpu.ids gpurun_out/r06h_enc_trace.txt | tail -18
