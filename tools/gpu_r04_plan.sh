#!/bin/bash
# Launch-plan sweep of the product build: launches in flight x batches per
# launch at the driver's 20 / 5 shape and at 48 / 16.
#   bash tools/gpu_r04_plan.sh <outdir> "inflight merge" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4plan}
shift
mkdir -p $O
cd $R
for cfg in "$@"; do
  set -- $cfg
  for sw in "20 5" "48 16"; do
    set -- $cfg $sw
    f=$O/i$1_m$2_s$3.json
    timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --inflight $1 --merge $2 --steps $3 --warmup $4 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));print('inflight $1 merge $2 steps $3', d['value'], d['ms_per_step'])"
  done
done
