#!/bin/bash
# Round-6 evidence at HEAD, part B: the side lines (48 steps, 1 % invalid,
# configs 5 / 3 / 4, config 4 through tbg_multi with its host share, the
# --gpus 2 launch on the one GPU) and the PMC traffic passes.
#   bash tools/gpu_r06_side.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r6side}
mkdir -p $O
cd $R
run() {  # name, bench flags...
  local n=$1; shift
  timeout -k 10 400 python3 -u bench.py --no-cpu --latency 0 "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n', d['value'], d['n_gpus'], d['config'].get('level0'), d['config'].get('rlc_group'), d.get('subgroup_batch'), d['roofline']['frac'] if d.get('roofline') else None)"
}
run s48 --steps 48 --warmup 16 --api-batches 0 || exit 1
run inject1 --steps 20 --warmup 5 --inject 0.01 --api-batches 0 || exit 1
run config5 --workload config5 --steps 20 --warmup 5 || exit 1
run config3 --workload config3 --steps 6 --warmup 2 || exit 1
run config4 --workload config4 --steps 4 --warmup 2 || exit 1
run gpus2 --gpus 2 --steps 20 --warmup 5 --api-batches 0 || exit 1
timeout -k 10 400 python3 -u bench.py --workload config4 --multi-contexts 8 --steps 3 --inject 0.01 > $O/bench_config4_multi.json 2> $O/bench_config4_multi.err || { tail -20 $O/bench_config4_multi.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_config4_multi.json'));print('config4_multi', d['value'], d['exact'], json.dumps(d['host_side']))"
bash tools/gpu_pmc.sh 16 && cp -r gpurun_out/pmc $O/pmc
