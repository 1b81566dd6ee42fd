#!/bin/bash
# Runtime A/B of an environment knob: default and driver-style (20/5) bench
# lines for each setting, alternated twice.  Usage: gpu_ab_env.sh VAR v1 v2
VAR=$1; A=$2; B=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abenv
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in $A $B; do
    for cfg in "48 16" "20 5"; do
      set -- $cfg
      f=$O/${VAR}_${v}_s$1_r$rep.json
      env $VAR=$v timeout -k 10 150 python bench.py --no-cpu --api-batches 0 --steps $1 --warmup $2 > $f 2> $f.err || { tail -3 $f.err; exit 1; }
      python3 -c "import json;d=json.load(open('$f'));print('$VAR=$v steps $1 rep $rep:', d['value'])"
    done
  done
done
