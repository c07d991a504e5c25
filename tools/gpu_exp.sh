set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 240 python bench.py --no-cpu --no-other --workload C5 "$@" > gpurun_out/s_$tag.json 2> gpurun_out/s_$tag.err || { echo "FAILED $tag"; tail -5 gpurun_out/s_$tag.err; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(sys.argv[2], d["value"], d["ms_per_step"], d["ms_per_step_serial"], r["launch_ms"], r["frac"], d["bit_exact"])' gpurun_out/s_$tag.json "$tag"; }
for rep in 1 2; do
for n in 512 256 128; do
 XA_STRIDE_BREAK=0 run n${n}_b0_$rep --streams $n --steps 20 --no-verify
 XA_STRIDE_BREAK=1 run n${n}_b1_$rep --streams $n --steps 20 --no-verify
done
done
XA_STRIDE_BREAK=1 run n512_b1_v --streams 512 --steps 5
