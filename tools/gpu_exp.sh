set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 240 python bench.py --no-cpu --no-other --no-verify --workload C5 "$@" > gpurun_out/q_$tag.json 2> gpurun_out/q_$tag.err || { echo "FAILED $tag"; tail -5 gpurun_out/q_$tag.err; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["ms_per_step"], d["ms_per_step_serial"], d["roofline"]["launch_ms"])' gpurun_out/q_$tag.json "$tag"; }
for rep in 1 2; do
for n in 512 256 128; do
 for d in 1 2; do run n${n}_d${d}_$rep --streams $n --steps 40 --pipeline $d; done
done
done
