#!/bin/bash
# Round-5 call: the level-1 group size on the invalid workloads (1 % invalid
# at the driver shape, config 5): the adaptive default (8 past 0.3 %
# invalid) against fixed 4, 8, 16.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r5grp
mkdir -p $O
run() {  # name args...
  local n=$1 f=$O/$1.json; shift
  timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 "$@" > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('$n', d['value'], d['config'].get('rlc_group'), d['fallback_levels'])"
}
for g in 0 4 8 16; do
  run inj_g$g --steps 20 --warmup 5 --inject 0.01 --rlc-group $g || exit 1
done
for g in 0 4 16; do
  run c5_g$g --workload config5 --steps 20 --warmup 5 --rlc-group $g || exit 1
done
