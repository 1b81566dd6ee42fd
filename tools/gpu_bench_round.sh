#!/bin/bash
# The round's bench evidence: the default bench line (CPU baseline included),
# the driver's usual invocation (--steps 20 --warmup 5), and a rocprofv3
# kernel-trace summary of the default bench (timed region included).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['ms_per_step'], d['roofline'], d['cpu_baseline'], d['api_pipeline'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_s20w5.json 2> $O/bench_s20w5.err || { tail -5 $O/bench_s20w5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_s20w5.json'));print('s20w5', d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --api-batches 0 > $O/bench_prof.json 2> $O/prof.log || { tail -5 $O/prof.log; exit 1; }
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:40]:40s} calls {r["Calls"]:>4s} avg_ms {float(r["AverageNs"])/1e6:8.3f}')
PY
