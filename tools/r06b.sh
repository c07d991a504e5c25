set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
timeout -k 10 120 python tools/clock_probe.py --rounds 10 > gpurun_out/r06b_clock.json 2> gpurun_out/r06b_clock.err || { echo clock failed; tail gpurun_out/r06b_clock.err; exit 1; }
cat gpurun_out/r06b_clock.json
timeout -k 10 180 tools/bin/write_probe2 > gpurun_out/r06b_write2.json 2>&1 || { echo write failed; tail gpurun_out/r06b_write2.json; exit 1; }
cat gpurun_out/r06b_write2.json
for mix in W A; do
timeout -k 10 300 python tools/ab_inproc.py --wl C3 --mix $mix --reps 5 w8=$L:0:0:8 w12=$L:0:0:12 w16=$L:0:0:16 w24=$L:0:0:24 > gpurun_out/r06b_wsweep_$mix.log 2>&1 || { echo ab failed; tail gpurun_out/r06b_wsweep_$mix.log; exit 1; }
cat gpurun_out/r06b_wsweep_$mix.log
done
