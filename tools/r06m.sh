# encode kernel: non-temporal XA stores (shipped) against plain ones
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in nt plain; do
if [ $v = plain ]; then export BJXA_LIB_PATH=$PWD/ab6/encplain/libbjxa.so.0; else unset BJXA_LIB_PATH; fi
timeout -k 10 120 python tools/encode_bench.py --steps 50 > gpurun_out/r06m.json 2>/dev/null || { echo failed; exit 1; }
echo "$v $(cat gpurun_out/r06m.json)"
done
done
