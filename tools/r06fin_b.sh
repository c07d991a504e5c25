# round-6 final evidence, part B: rocprofv3 trace + counter passes of the
# bench (100 steps), and the trace of the same command one step at a time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${1:-r06fin}
bash tools/gpu_run.sh $T "prof=--steps 100" || exit 1
mkdir -p gpurun_out/prof_${T}_serial
( export TMPDIR=/tmp; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OLDPWD/gpurun_out/prof_${T}_serial" -o run -- python3 "$OLDPWD/bench.py" --steps 100 --pipeline 1 \
    > "$OLDPWD/gpurun_out/prof_${T}_serial/bench.json" 2> "$OLDPWD/gpurun_out/prof_${T}_serial/trace.log" ) || { echo serial trace failed; exit 1; }
echo serial done
