#!/bin/bash
# Kernel trace of the injected-invalid workload (one launch in flight, so the
# per-kernel times are exclusive).  Output under gpurun_out/ab/<tag>/.
TAG=${1:-inject}
RATE=${2:-0.01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_inject -o run -- python3 $R/bench.py --no-cpu --inflight 1 --steps 4 --warmup 1 --api-batches 0 --inject $RATE > $O/prof_inject.json 2> $O/prof_inject.log || { tail -5 $O/prof_inject.log; exit 1; }
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/prof_inject/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    print(f'{r["Name"][:40]:40s} calls {r["Calls"]:>4s} avg_ms {float(r["AverageNs"])/1e6:8.3f}')
PY
