#!/bin/bash
# Uneven launch sizes for the driver's 20-step run:  bash tools/gpu_r04_split.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4split}
mkdir -p $O
cd $R
for sp in "7,7,6" "9,7,4" "10,6,4" "8,7,5" "11,6,3" "7,7,6"; do
  f=$O/split_${sp//,/_}_$RANDOM.json
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --split $sp --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('split $sp', d['value'])"
done
