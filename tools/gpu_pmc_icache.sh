#!/bin/bash
# One SQ counter pass (8 SQ counters) for the instruction cache: requests,
# hits, misses, fetches against wave cycles / issue stalls / VALU issue, over
# one launch of M batches (kernels serialised by the counter collection).
#   bash tools/gpu_pmc_icache.sh [M] [outdir] [extra bench.py args]
M=${1:-16}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${2:-icache}
shift 2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -f csv -d $O/pmc -o run -- python3 $R/bench.py --no-cpu --inflight 1 --merge $M --steps $M --warmup 0 --api-batches 0 --latency 0 "$@" > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
cd $R && python3 - $O/pmc/run_counter_collection.csv <<'PY'
import csv, collections, sys
d = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tbg::", "")
    d[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:20]:
    req = v["SQC_ICACHE_REQ"] or 1
    wc = v["SQ_WAVE_CYCLES"] or 1
    print(f"{k[:34]:34s} wave_cyc {wc:.3g} miss/req {v['SQC_ICACHE_MISSES']/req:.4f} dup/req {v['SQC_ICACHE_MISSES_DUPLICATE']/req:.4f} "
          f"hit/req {v['SQC_ICACHE_HITS']/req:.4f} ifetch {v['SQ_IFETCH']:.3g} wait_inst/wc {4*v['SQ_WAIT_INST_ANY']/wc:.3f} valu/wc {4*v['SQ_ACTIVE_INST_VALU']/wc:.3f}")
PY
