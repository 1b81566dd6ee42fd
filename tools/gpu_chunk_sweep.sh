#!/bin/bash
# Level-0 schedule knobs: duties per Miller quad (rlc_chunk) and per group.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chunk
mkdir -p $O
cd $R
for cfg in "16 4" "16 3" "15 5" "32 4" "16 8"; do
  set -- $cfg
  f=$O/g$1_c$2.json
  timeout -k 10 150 python bench.py --no-cpu --api-batches 0 --rlc-group $1 --rlc-chunk $2 > $f 2> $f.err || { tail -3 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('group $1 chunk $2:', d['value'], d['config']['level0'], d['isolated_batch_ms']['verify'])"
done
