#!/bin/bash
# Launch-plan sweep: the same timed steps spread over different launch counts
# (and slots in flight).  Output: gpurun_out/plan/<tag>_s<steps>_L<launches>_i<inflight>.json
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/plan
mkdir -p $O
cd $R
for cfg in "20 5 3 3" "20 5 4 3" "20 5 5 3" "20 5 6 3" "20 5 5 4" "20 5 10 4" "48 16 3 3" "48 16 6 3" "48 16 4 4"; do
  set -- $cfg
  f=$O/s$1_w$2_L$3_i$4.json
  timeout -k 10 150 python bench.py --no-cpu --api-batches 0 --steps $1 --warmup $2 --launches $3 --inflight $4 > $f 2> $f.err || { tail -3 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('steps $1 launches $3 inflight $4:', d['value'], d['ms_per_step'])"
done
