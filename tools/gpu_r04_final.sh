#!/bin/bash
# Round-4 evidence at HEAD, first call: the GPU suite, smoke(), and the
# driver's bench command under a rocprofv3 kernel trace.
#   bash tools/gpu_r04_final.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r4final}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_r04_tests.sh $D || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
bash tools/gpu_r04_bench.sh $D A
