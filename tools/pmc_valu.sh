#!/bin/bash
# VALU utilisation pass (run on the box through gpurun): lists the gfx950
# SQ counters, then collects VALU instruction / active-cycle counters for one
# isolated 10k-DV batch chain (--inflight 1) in a pass of its own (no trace
# domains beside --pmc; at most 8 SQ + 2 GRBM counters per pass).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/valu
mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" $O/counters.txt | sort -u > $O/sq_counters.txt || true
C="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for x in SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64; do
  if grep -qx "$x" $O/sq_counters.txt; then C="$C $x"; fi
done
echo "counters: $C"
timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $O/pmc -o run -- python3 $R/bench.py --no-cpu --steps 4 --inflight 1 > $O/pmc.log 2>&1
echo "== done"
