#!/bin/bash
# Quick A/B: optional microbench, then the driver's bench command (20/5) twice.
#   bash tools/gpu_r03_quick.sh <outdir> [extra bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3q}
shift
mkdir -p $O
cd $R
if [ -x tools/microbench/wide_fe_bench ]; then
  timeout -k 10 60 tools/microbench/wide_fe_bench > $O/wide_fe.txt 2>&1 || { cat $O/wide_fe.txt; exit 1; }
  cat $O/wide_fe.txt
fi
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 "$@" > $O/bench_s20_$i.json 2> $O/bench_s20_$i.err || { tail -20 $O/bench_s20_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_s20_$i.json'));print('s20', d['value'], d['config']['level0'], d['roofline']['kernel'], d['roofline']['frac'])"
done
