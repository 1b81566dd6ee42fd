#!/bin/bash
# Kernel trace of the driver-style run (20 steps, 5 warmup): per-kernel
# intervals of the timed region for the idle-time analysis (tools/timeline.py).
#   bash tools/gpu_trace20.sh [outdir] [extra bench.py args, e.g. --inject 0.01]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-trace20}
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --api-batches 0 --steps 20 --warmup 5 "$@" > $O/bench.json 2> $O/prof.log || { tail -5 $O/prof.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'])"
