#!/bin/bash
# Isolated per-kernel evidence for the current build: a kernel-trace of one
# launch in flight (exclusive kernel times) and the two PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE; separate runs), all on launches of M batches.
M=${1:-16}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu --inflight 1 --merge $M --steps $((2*M)) --warmup 0 --api-batches 0 --latency 0 > $O/trace.json 2> $O/trace.log || { tail -5 $O/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu --inflight 1 --merge $M --steps $M --warmup 0 --api-batches 0 --latency 0 > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu --inflight 1 --merge $M --steps $M --warmup 0 --api-batches 0 --latency 0 > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; exit 1; }
cd $R && python3 tools/pmc_traffic.py $O $O/traffic.json $M && python3 - <<PY
import csv, json
rows = list(csv.DictReader(open("$O/trace/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:40]:40s} calls {r["Calls"]:>4s} avg_ms {float(r["AverageNs"])/1e6:8.3f}')
t = json.load(open("$O/traffic.json"))["kernels"]
for k, v in sorted(t.items(), key=lambda kv: -kv[1].get("WRITE_SIZE_KB_per_launch", 0))[:10]:
    print(k, v)
PY
