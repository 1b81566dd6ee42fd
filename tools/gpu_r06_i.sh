#!/bin/bash
# Round-6 call I: group size under invalid traffic with level 1 on group
# MSMs: 1 % invalid at G = 4 / 8 (adaptive) / 16 and level 1g, config 5 at
# G = 8 / 16 (adaptive), interleaved twice.
#   bash tools/gpu_r06_i.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6i}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
for rep in 1 2; do
  for wl in "inj_auto:--inject 0.01" "inj_g4:--inject 0.01 --rlc-group 4" "inj_g16:--inject 0.01 --rlc-group 16" "inj_gid:--inject 0.01 --gident 1" "c5_auto:--workload config5" "c5_g8:--workload config5 --rlc-group 8"; do
    tag=${wl%%:*}; args=${wl#*:}
    f=$O/${tag}_$rep.json
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));print('$tag $rep', d['value'], d['config']['rlc_group'], d['isolated_batch_ms']['total'], d['fallback_levels'])"
  done
done
