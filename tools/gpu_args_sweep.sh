#!/bin/bash
# One bench line per argument set (each argument set is one quoted string),
# under gpurun_out/argsweep/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/argsweep
mkdir -p $O
cd $R
k=0
for spec in "$@"; do
  k=$((k+1))
  timeout -k 10 240 python bench.py --no-cpu --api-batches 0 $spec > $O/run$k.json 2> $O/run$k.err || { echo "fail [$spec]"; tail -3 $O/run$k.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/run$k.json'));print('[$spec]', d['value'], d['ms_per_step'])"
done
