#!/bin/bash
# Bench the default launch shape with each library given (TBG_LIB), one line each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ablibs
mkdir -p $O
cd $R
for lib in "$@"; do
  n=$(basename $lib .so)
  TBG_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu --api-batches 0 > $O/$n.json 2> $O/$n.err || { echo "fail $n"; tail -3 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['isolated_batch_ms'], d['roofline']['frac'], d['roofline_isolated']['frac'])"
done
