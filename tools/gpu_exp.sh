set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 240 python bench.py --no-cpu --no-other --no-verify "$@" > gpurun_out/w_$tag.json 2> gpurun_out/w_$tag.err || { echo "FAILED $tag"; tail -5 gpurun_out/w_$tag.err; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(sys.argv[2], d["value"], d["ms_per_step"], d["ms_per_step_serial"], r["launch_ms"], d["repaired_chunks"])' gpurun_out/w_$tag.json "$tag"; }
for rep in 1 2; do
for mix in A W F; do
for wc in 8:40 6:40 4:40 8:36 4:36; do
 w=${wc%:*}; c=${wc#*:}
 run ${mix}_w${w}_c${c}_$rep --mix $mix --warm-blocks $w --chunk $c --steps 100
done
done
done
