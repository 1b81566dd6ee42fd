#!/bin/bash
# Quick A/B pass for a kernel change: the fixture + oracle parity subset, one
# bench line (no CPU leg) and a rocprofv3 kernel-trace of one batch in flight
# (exclusive kernel times).  Output under gpurun_out/ab/<tag>/.  Stops at the
# first failure.
TAG=${1:-ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or kat or config5 or config2 or cancelling" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench.py --no-cpu --api-batches 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['isolated_batch_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --inflight 1 --steps 4 --warmup 1 --api-batches 0 > $O/prof.json 2> $O/prof.log || { tail -5 $O/prof.log; exit 1; }
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:40]:40s} calls {r["Calls"]:>4s} avg_ms {float(r["AverageNs"])/1e6:8.3f}')
PY
