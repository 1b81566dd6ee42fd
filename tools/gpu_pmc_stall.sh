#!/bin/bash
# One SQ counter pass (8 SQ counters: the most one pass may hold) over one
# launch of M batches in flight: wave time split into memory waits, issue
# stalls and issue (tools/pmc_stall.py).
#   bash tools/gpu_pmc_stall.sh [M] [outdir] [extra bench.py args, e.g. --inject 0.01]
M=${1:-16}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${2:-stall}
shift 2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -f csv -d $O/pmc -o run -- python3 $R/bench.py --no-cpu --inflight 1 --merge $M --steps $M --warmup 0 --api-batches 0 --latency 0 "$@" > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
cd $R && python3 tools/pmc_stall.py $O/pmc/run_counter_collection.csv $O/stall.json
