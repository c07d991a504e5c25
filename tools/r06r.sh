set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for rep in 1 2 3; do
for p in 2 3; do
timeout -k 10 300 python bench.py --workload C3 --no-other --no-cpu --no-verify --steps 100 --pipeline $p > gpurun_out/r06r.json 2>/dev/null || { echo failed; exit 1; }
python -c "import json,sys; L=[l for l in open(sys.argv[1]) if l.startswith('{')][-1]; d=json.loads(L); print('pipeline', $p, d['ms_per_step'], d['ms_per_step_serial'], d['roofline']['launch_ms'])" gpurun_out/r06r.json
done
done
