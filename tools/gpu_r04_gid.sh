#!/bin/bash
# Level-1g routing at 1 % invalid (20 / 5 and 48 / 16) and config 5:
#   bash tools/gpu_r04_gid.sh <outdir> <gident values ...>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4gid}
shift
mkdir -p $O
cd $R
for g in "$@"; do
  for sw in "20 5" "48 16"; do
    set -- $sw
    f=$O/g${g}_inject1_s$1.json
    timeout -k 10 400 python3 -u bench.py --steps $1 --warmup $2 --inject 0.01 --gident $g --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));print('gident $g inject1 steps $1', d['value'], d['fallback_levels'])"
  done
  f=$O/g${g}_config5.json
  timeout -k 10 400 python3 -u bench.py --workload config5 --steps 20 --warmup 5 --gident $g --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('gident $g config5', d['value'])"
done
