#!/bin/bash
# Round-3 measurement: the driver's bench command under a rocprofv3 kernel
# trace (+ the roofline recomputed from that trace), then the side lines.
#   bash tools/gpu_r03_bench.sh <outdir> [headline|side]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3bench}
WHAT=${2:-headline}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ "$WHAT" = headline ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20w5.json 2> $O/bench_s20w5.err || { tail -20 $O/bench_s20w5.err; exit 1; }
  cd $R && python3 tools/roofline_from_trace.py $O/prof/run_kernel_trace.csv $O/bench_s20w5.json --out $O/roofline_check.json
else
  cd $R
  timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --inject 0.01 --no-cpu --api-batches 0 > $O/bench_inject1.json 2> $O/bench_inject1.err || { tail -20 $O/bench_inject1.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --workload config5 --steps 20 --warmup 5 --no-cpu > $O/bench_config5.json 2> $O/bench_config5.err || { tail -20 $O/bench_config5.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --workload config3 --steps 6 --warmup 2 --cpu-seconds 10 > $O/bench_config3.json 2> $O/bench_config3.err || { tail -20 $O/bench_config3.err; exit 1; }
  for f in inject1 config5 config3; do python3 -c "import json;d=json.load(open('$O/bench_$f.json'));print('$f', d['value'], d['config']['level0'], d['roofline']['kernel'], d['roofline']['frac'])"; done
fi
