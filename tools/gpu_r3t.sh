#!/bin/bash
# N > 1 path on the final build: the C5 line at one rank through RCCL
# (--force-pg), and the gloo-gpu rehearsal of the 8-rank job on GPU 0
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 300 python bench.py --gpus 1 --force-pg --workload C5 --steps 20 > gpurun_out/r3/c5_rccl1.json 2> gpurun_out/r3/c5_rccl1.err || { tail -20 gpurun_out/r3/c5_rccl1.err; exit 1; }
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("checksums_match_oracle"), d["config"].get("parallelism"))' gpurun_out/r3/c5_rccl1.json
BJXA_BENCH_BACKEND=gloo-gpu timeout -k 10 600 python bench.py --gpus 8 --steps 5 --warmup 1 > gpurun_out/r3/c5_gloo8.json 2> gpurun_out/r3/c5_gloo8.err || { tail -20 gpurun_out/r3/c5_gloo8.err; exit 1; }
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["n_gpus"], d["value"], d.get("checksums_match_oracle"), d.get("bit_exact"))' gpurun_out/r3/c5_gloo8.json
