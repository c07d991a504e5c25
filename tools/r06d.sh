# C4: the balanced grid order of batch waves against stream order (bit 21)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_c5.py tests/test_gpu_files.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06d_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r06d_tests.log; exit 1; }
tail -2 gpurun_out/r06d_tests.log
for wl in C4 C5g; do
timeout -k 10 300 python tools/ab_inproc.py --wl $wl --reps 6 stream=$L spread=$L:0x400000 cluster=$L:0x800000 > gpurun_out/r06d_ab_$wl.log 2>&1 || { echo "ab $wl failed"; tail gpurun_out/r06d_ab_$wl.log; exit 1; }
echo "== $wl"; grep -v amdgpu.ids gpurun_out/r06d_ab_$wl.log
done


timeout -k 10 180 tools/bin/zc_probe > gpurun_out/r06d_zc.json 2>&1 || { echo "zc failed"; tail gpurun_out/r06d_zc.json; exit 1; }
grep -E "duplex|register" gpurun_out/r06d_zc.json
