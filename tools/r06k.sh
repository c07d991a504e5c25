# K1's prologue landing both halves of super-step 0 at once (new) against
# the previous build (ab6/pre), interleaved in one process
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_settle.py tests/test_gpu_batch.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06k_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r06k_tests.log; exit 1; }
tail -1 gpurun_out/r06k_tests.log
for wl in C3 C2 C5g C4; do
timeout -k 10 400 python tools/ab_inproc.py --wl $wl --reps 8 new=bjxa_amd/libbjxa.so.0 pre=ab6/pre/libbjxa.so.0 > gpurun_out/r06k_ab_$wl.log 2>&1 || { echo ab failed; tail gpurun_out/r06k_ab_$wl.log; exit 1; }
echo "== $wl"; grep -v amdgpu.ids gpurun_out/r06k_ab_$wl.log
done
