#!/bin/bash
# rlc_chunk 4 vs 8 at level 0, 48 and 20 steps, alternated twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chunkab
mkdir -p $O
cd $R
for rep in 1 2; do
  for c in 4 8 6; do
    for st in "48 16" "20 5"; do
      set -- $st
      f=$O/c${c}_s$1_r$rep.json
      timeout -k 10 150 python bench.py --no-cpu --api-batches 0 --rlc-chunk $c --steps $1 --warmup $2 > $f 2> $f.err || { tail -3 $f.err; exit 1; }
      python3 -c "import json;d=json.load(open('$f'));print('chunk $c steps $1 rep $rep:', d['value'])"
    done
  done
done
