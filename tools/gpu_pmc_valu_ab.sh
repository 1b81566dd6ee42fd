#!/bin/bash
# SQ counters of the level-0 Miller kernel (one launch of 16 batches in
# flight) for several builds / knobs:  bash tools/gpu_pmc_valu_ab.sh <outdir> VAR=a ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-valuab}
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
for kv in "$@"; do
  n=$(echo "$kv" | tr '/=' '__')
  export $(echo "$kv" | sed "s|=varlib/|=$R/varlib/|")
  timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $O/$n -o run -- python3 $R/bench.py --no-cpu --inflight 1 --merge 16 --steps 16 --warmup 0 --api-batches 0 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  unset ${kv%%=*}
  python3 - "$O/$n/run_counter_collection.csv" "$kv" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "miller" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[2], {k: int(v) for k, v in sorted(agg.items())})
if agg.get("SQ_WAVE_CYCLES"):
    print("   valu/wavecyc", round(agg["SQ_ACTIVE_INST_VALU"] / agg["SQ_WAVE_CYCLES"], 3),
          "wait_any", round(agg["SQ_WAIT_ANY"] / agg["SQ_WAVE_CYCLES"], 3),
          "wait_inst", round(agg["SQ_WAIT_INST_ANY"] / agg["SQ_WAVE_CYCLES"], 3),
          "insts/wave", int(agg["SQ_INSTS_VALU"] / max(1, agg["SQ_WAVES"])))
PY
done
