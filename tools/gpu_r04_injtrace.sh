#!/bin/bash
# Kernel trace of one launch (16 batches) at 1 % invalid: per-dispatch
# durations of the fallback levels (tools/iso_from_trace.py style summary).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-injtrace}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu --inflight 1 --merge 16 --steps 16 --warmup 0 --api-batches 0 --inject 0.01 > $O/trace.json 2> $O/trace.log || { tail -5 $O/trace.log; exit 1; }
cd $R && python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$O/trace/run_kernel_trace.csv")))
per = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("tbg::", "").replace("void ", "")
    per[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for n in ("k_rlc_group_final", "k_rlc_check_chunks", "k_rlc_cident_check", "k_rlc_ident_check", "k_verify_list",
          "k_lines_fold<FOLD_CHUNKS>", "k_rlc_chunk_lines", "k_l0_final", "k_l0_inv", "k_l0_fe"):
    v = per.get(n, [])
    print(n, len(v), [round(x, 3) for x in sorted(v, reverse=True)[:8]])
PY
