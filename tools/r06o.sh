set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for rep in 1 2 3 4; do
for cfg in "64 128" "192 384" "224 448"; do
set -- $cfg
for ch in 2 1; do
BJXA_DUPLEX_OUT_CUS=$1 BJXA_DUPLEX_OUT_WGS=$2 timeout -k 10 120 python tools/host_rate.py --ch $ch --passes 5 > gpurun_out/r06o.json 2>/dev/null || { echo failed; exit 1; }
echo "cus=$1 wgs=$2 ch=$ch $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms'], d['bit_exact'])" gpurun_out/r06o.json)"
done
done
done
