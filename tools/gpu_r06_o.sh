#!/bin/bash
# Round-6 call O: the 20-step plan's launch sizes (7+7+6 default vs
# descending splits), three reps interleaved on one box.
#   bash tools/gpu_r06_o.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6o}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for sp in default 8,7,5 9,7,4 8,8,4 10,6,4; do
    if [ $sp = default ]; then extra=""; else extra="--split $sp"; fi
    f=$O/plan_${sp//,/_}_$rep.json
    timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 --steps 20 --warmup 5 $extra > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$f'));print('$sp $rep', d['value'])"
  done
done
