# Duplex slabs of 8 MiB with decode groups to 8 (oldlib/, built with
# -DDUPLEX_SLAB_MIB=8 -DDUPLEX_GROUP=8) against the shipped 16 MiB / 4:
# duplex tests on the variant, then alternating fresh processes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
BJXA_LIB_PATH=oldlib/libbjxa.so.0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_duplex.py > gpurun_out/r06z19_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06z19_tests.txt; exit 1; }
tail -1 gpurun_out/r06z19_tests.txt
for i in 1 2 3; do
for ch in 2 1; do
echo "slab8 ch=$ch $(BJXA_LIB_PATH=oldlib/libbjxa.so.0 timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-140)" || exit 1
echo "slab16 ch=$ch $(timeout -k 10 200 python tools/host_rate.py --ch $ch --passes 9 | cut -c1-140)" || exit 1
done
done
echo "slab8 enc $(BJXA_LIB_PATH=oldlib/libbjxa.so.0 timeout -k 10 200 python tools/host_rate.py --encode --ch 2 --passes 9 | cut -c1-140)" || exit 1
echo "slab16 enc $(timeout -k 10 200 python tools/host_rate.py --encode --ch 2 --passes 9 | cut -c1-140)" || exit 1
