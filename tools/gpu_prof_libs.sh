#!/bin/bash
# Kernel traces of one batch per launch (exclusive kernel times) for each
# library given (TBG_LIB); per-kernel averages side by side.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/proflibs
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  TBG_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 $R/bench.py --no-cpu --merge 1 --inflight 1 --steps 6 --warmup 2 --api-batches 0 ${PROF_ARGS} > $O/$n.json 2> $O/$n.log || { tail -5 $O/$n.log; exit 1; }
done
python3 - "$O" "$@" <<'PY'
import csv, os, sys
o, libs = sys.argv[1], [os.path.basename(l)[:-3] for l in sys.argv[2:]]
tabs = [{r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(f"{o}/{n}/run_kernel_stats.csv"))} for n in libs]
for k in sorted(set().union(*tabs)):
    if k.startswith("tbg::k_sign") or k.startswith("tbg::k_sk"): continue
    print(f"{k[5:40]:36s}" + "".join(f"{t.get(k, 0):9.3f}" for t in tabs))
PY
