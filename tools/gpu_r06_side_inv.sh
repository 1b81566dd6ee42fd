#!/bin/bash
# The invalid-traffic side lines at the driver shape: 1 % invalid partials
# and config 5 (mixed duties / thresholds, every injection kind).
#   bash tools/gpu_r06_side_inv.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r6side}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 --steps 20 --warmup 5 --inject 0.01 > $O/inv1.json 2> $O/inv1.err || { tail -20 $O/inv1.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 --steps 20 --warmup 5 --workload config5 > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
for n in inv1 config5; do
  python3 -c "
import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], [x['exact'] for x in d['ranks_exact_after_clock']])"
done
