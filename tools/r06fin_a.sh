# round-6 final evidence, part A: GPU suite, smoke, the driver's bench
# command, the 8-rank gloo rehearsal and the RCCL control plane at one rank
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${1:-r06fin}
bash tools/gpu_run.sh $T tests smoke "bench=--steps 20 --warmup 5" || exit 1
BJXA_BENCH_BACKEND=gloo-gpu timeout -k 10 600 python bench.py --gpus 8 --steps 5 --warmup 2 --no-cpu > gpurun_out/${T}_rehearsal8.json 2> gpurun_out/${T}_rehearsal8.err || { echo rehearsal failed; tail -20 gpurun_out/${T}_rehearsal8.err; exit 1; }
tail -c 400 gpurun_out/${T}_rehearsal8.json; echo
timeout -k 10 300 python bench.py --gpus 1 --force-pg --workload C5 --steps 10 --no-cpu > gpurun_out/${T}_rccl1.json 2> gpurun_out/${T}_rccl1.err || { echo rccl failed; tail -20 gpurun_out/${T}_rccl1.err; exit 1; }
tail -c 400 gpurun_out/${T}_rccl1.json; echo
