set -o pipefail
mkdir -p gpurun_out
bash tools/trace.sh c5 --workload C5 --steps 20 || exit 1
bash tools/trace.sh c5n8 --workload C5 --streams 128 --steps 50 || exit 1
bash tools/trace.sh c5n2 --workload C5 --streams 512 --steps 20 || exit 1
for t in c5 c5n8 c5n2; do python3 tools/pmc_summary.py gpurun_out/prof_$t --json gpurun_out/prof_$t/summary.json > /dev/null; python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k: v for k, v in d["kernel_us_alone"].items() if "xa_" in k}, {k: v for k, v in d["kernel_us"].items() if "xa_" in k})' gpurun_out/prof_$t/summary.json; done
