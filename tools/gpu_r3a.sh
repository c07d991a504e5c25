cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_large.py > gpurun_out/r3/t1.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 gpurun_out/r3/t1.log
if [ $rc -le 1 ]; then
  timeout -k 10 240 python -u tools/ab_inproc.py --wl C3 --reps 4 region=bjxa_amd/libbjxa.so.0:128 strided=bjxa_amd/libbjxa.so.0:0 > gpurun_out/r3/ab1.log 2>&1
  echo "ab rc=$?"
  tail -8 gpurun_out/r3/ab1.log
fi
