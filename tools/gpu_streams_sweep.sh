#!/bin/bash
# Slots x streams-per-slot sweep at 48 and 20 steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/streams
mkdir -p $O
cd $R
for cfg in "3 1" "2 2" "3 2" "4 1"; do
  set -- $cfg
  for st in "48 16" "20 5"; do
    set -- $cfg $st
    f=$O/i$1_s$2_steps$3.json
    timeout -k 10 150 python bench.py --no-cpu --api-batches 0 --inflight $1 --streams-per-slot $2 --steps $3 --warmup $4 > $f 2> $f.err || { tail -3 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));print('inflight $1 streams $2 steps $3:', d['value'])"
  done
done
