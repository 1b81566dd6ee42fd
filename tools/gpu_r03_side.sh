#!/bin/bash
# Round-3 side measurements at HEAD: 48-step headline, 1 % invalid, config 5,
# config 3, then the PMC traffic passes (tools/gpu_pmc.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3side}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --steps 48 --warmup 16 --no-cpu --api-batches 0 > $O/bench_s48.json 2> $O/bench_s48.err || { tail -20 $O/bench_s48.err; exit 1; }
bash tools/gpu_r03_bench.sh ${1:-r3side} side || exit 1
bash tools/gpu_pmc.sh 16 || exit 1
