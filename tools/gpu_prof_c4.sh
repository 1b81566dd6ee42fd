#!/bin/bash
# Per-kernel times on a config-4 shard (125k DVs: every stage fills the GPU):
# rocprofv3 kernel-trace of one batch in flight, plus the config-4 bench line.
TAG=${1:-c4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c4/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --workload config4 --no-cpu --inflight 1 --steps 3 --warmup 1 --api-batches 0 > $O/bench.json 2> $O/prof.log || { tail -5 $O/prof.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['isolated_batch_ms'])"
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:40]:40s} calls {r["Calls"]:>4s} avg_ms {float(r["AverageNs"])/1e6:8.3f}')
PY
