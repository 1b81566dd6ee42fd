#!/bin/bash
# Injected-invalid throughput at several launch depths (and the clean rate
# at the same depths), one JSON line each under gpurun_out/ab/<tag>/.
TAG=${1:-sweep}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab/$TAG
mkdir -p $O
cd $R
for spec in "$@"; do   # spec = inflight:inject
  i=${spec%%:*}; r=${spec##*:}
  timeout -k 10 200 python bench.py --no-cpu --api-batches 0 --inflight $i --inject $r > $O/i${i}_r${r}.json 2> $O/i${i}_r${r}.err || { tail -3 $O/i${i}_r${r}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/i${i}_r${r}.json'));print('inflight $i inject $r', d['value'], d['ms_per_step'])"
done
