#!/bin/bash
# Bench lines for each library (TBG_LIB) x launch shape: specs are
# lib:inflight:inject:merge.  Output under gpurun_out/libsweep/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/libsweep
mkdir -p $O
cd $R
for spec in "$@"; do
  IFS=: read lib i r m <<< "$spec"
  n=$(basename $lib .so)_i${i}_r${r}_m${m}
  TBG_LIB=$R/$lib timeout -k 10 240 python bench.py --no-cpu --api-batches 0 --inflight $i --inject $r --merge $m > $O/$n.json 2> $O/$n.err || { echo "fail $n"; tail -3 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'])"
done
