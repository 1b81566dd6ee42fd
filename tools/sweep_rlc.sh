#!/bin/bash
# Bench at several RLC group / chunk sizes (duties per level-1 group, duties per Miller quad).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sweep_rlc
mkdir -p $O
cd $R
for cfg in "8 2" "8 4" "16 2" "16 4" "16 8" "32 4"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu --rlc-group $1 --rlc-chunk $2 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -5 $O/b_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$1_$2.json'));print('group',$1,'chunk',$2,d['value'],d['isolated_batch_ms']['verify'])"
done
