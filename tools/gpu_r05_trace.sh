#!/bin/bash
# rocprofv3 kernel trace of one bench command + the timed region's timeline
# (tools/timeline.py): which chains run where, and the idle stretches.
#   bash tools/gpu_r05_trace.sh <outdir> [bench flags...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5trace}
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 --latency 0 "$@" > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cd $R && python3 tools/timeline.py $O/trace/run_kernel_trace.csv > $O/timeline.txt 2>&1 || { tail -5 $O/timeline.txt; exit 1; }
head -3 $O/timeline.txt
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value', d['value'], d['config']['level0'], d['config']['rlc_group'])"
