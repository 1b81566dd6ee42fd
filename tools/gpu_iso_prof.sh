#!/bin/bash
# Exclusive per-kernel times of full 16-batch launches (one launch in flight:
# initial submit, warmup, timed and isolated passes are all 16-batch launches)
# plus the driver-style short run (--steps 20 --warmup 5).  Extra bench
# arguments (e.g. --rlc-group 32) go to every run.  Output: gpurun_out/iso/<tag>/.
TAG=${1:-iso}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/iso/$TAG
mkdir -p $O
cd $R
timeout -k 10 200 python bench.py --no-cpu --api-batches 0 "$@" > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('default',d['value'],d['ms_per_step'],d['config']['rlc_group'])"
timeout -k 10 200 python bench.py --no-cpu --api-batches 0 --steps 20 --warmup 5 "$@" > $O/bench_s20.json 2> $O/bench_s20.err || { tail -5 $O/bench_s20.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_s20.json'));print('s20w5',d['value'],d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --inflight 1 --merge 16 --steps 16 --warmup 16 --api-batches 0 "$@" > $O/prof.json 2> $O/prof.log || { tail -5 $O/prof.log; exit 1; }
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:26]:
    print(f'{r["Name"][:40]:40s} calls {r["Calls"]:>4s} avg_ms {float(r["AverageNs"])/1e6:8.3f}')
PY
