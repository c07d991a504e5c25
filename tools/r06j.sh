set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
timeout -k 10 600 python -u -m pytest tests/test_gpu_duplex.py tests/test_gpu_threads.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06j_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r06j_tests.log; exit 1; }
tail -1 gpurun_out/r06j_tests.log
timeout -k 10 400 python tools/ab_inproc.py --wl C4 --reps 5 cb192=$L cb160=$L:0:160 cb128=$L:0:128 cb96=$L:0:96 cb224=$L:0:224 cb256=$L:0:256 > gpurun_out/r06j_c4_budget.log 2>&1 || { echo ab failed; tail gpurun_out/r06j_c4_budget.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06j_c4_budget.log
