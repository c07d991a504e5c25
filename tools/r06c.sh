# C5g (one rank's share of C5 at N = 8) against its placement, and the
# shares of N = 1/2/4/8 as bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
for lay in sep hipmalloc packed gaps pages; do
	timeout -k 10 300 python tools/ab_inproc.py --wl C5g --reps 5 --layout $lay new=$L new64=$L:0x20000 new68=$L:0x10000 > gpurun_out/r06c_c5g_$lay.log 2>&1 || { echo "ab $lay failed"; tail gpurun_out/r06c_c5g_$lay.log; exit 1; }
	echo "== $lay"; grep -v amdgpu.ids gpurun_out/r06c_c5g_$lay.log
done
for i in 1 2 3 4; do
	timeout -k 10 300 python bench.py --workload C5 --streams 128 --no-cpu --no-other --steps 20 > gpurun_out/r06c_c5g_fresh$i.json 2> gpurun_out/r06c_c5g_fresh$i.err || { echo "fresh $i failed"; tail gpurun_out/r06c_c5g_fresh$i.err; exit 1; }
	python -c "import json,sys; d=json.load(open(sys.argv[1])); print('fresh', d.get('ms_per_step'), d.get('ms_per_step_serial'), d['roofline'].get('launch_ms') if 'roofline' in d else d.get('spec_ms'))" gpurun_out/r06c_c5g_fresh$i.json
done
for S in 1024 512 256 128; do
	timeout -k 10 300 python bench.py --workload C5 --streams $S --no-cpu --no-other --steps 10 > gpurun_out/r06c_shard_$S.json 2> gpurun_out/r06c_shard_$S.err || { echo "shard $S failed"; tail gpurun_out/r06c_shard_$S.err; exit 1; }
done

timeout -k 10 180 tools/bin/zc_probe > gpurun_out/r06c_zc.json 2>&1 || { echo "zc failed"; tail gpurun_out/r06c_zc.json; exit 1; }
cat gpurun_out/r06c_zc.json
echo done
