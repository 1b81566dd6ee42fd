#!/bin/bash
# Group / chunk size at 1 % invalid (20 / 5) and on config 5:
#   bash tools/gpu_r04_grp.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4grp}
mkdir -p $O
cd $R
for gc in "8 4" "4 4" "4 2" "8 2" "16 4"; do
  set -- $gc
  f=$O/inj_g$1_c$2.json
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --inject 0.01 --rlc-group $1 --rlc-chunk $2 --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('inject1 group $1 chunk $2', d['value'], d['fallback_levels'])"
done
for gc in "16 4" "8 4" "4 4"; do
  set -- $gc
  f=$O/c5_g$1_c$2.json
  timeout -k 10 300 python3 -u bench.py --workload config5 --steps 20 --warmup 5 --rlc-group $1 --rlc-chunk $2 --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('config5 group $1 chunk $2', d['value'], d['fallback_levels'])"
done
