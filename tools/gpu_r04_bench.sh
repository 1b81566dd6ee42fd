#!/bin/bash
# Round-4 measurement at HEAD: the driver's bench command under a rocprofv3
# kernel trace (+ the roofline recomputed from that trace), then (part B)
# the side lines and the PMC traffic passes.
#   bash tools/gpu_r04_bench.sh <outdir> [A|B|AB]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4bench}
WHAT=${2:-AB}
mkdir -p $O
if [[ $WHAT == *A* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20w5.json 2> $O/bench_s20w5.err || { tail -20 $O/bench_s20w5.err; exit 1; }
  cd $R && python3 tools/roofline_from_trace.py $O/prof/run_kernel_trace.csv $O/bench_s20w5.json --out $O/roofline_check.json || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_s20w5.json'));print('s20', d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline'].get('frac_fp300'), d['roofline']['traffic'], d['api_pipeline']['value'] if d['api_pipeline'] else None)"
fi
if [[ $WHAT == *B* ]]; then
  cd $R
  timeout -k 10 300 python3 -u bench.py --steps 48 --warmup 16 --no-cpu --api-batches 0 > $O/bench_s48.json 2> $O/bench_s48.err || { tail -20 $O/bench_s48.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --inject 0.01 --no-cpu --api-batches 0 > $O/bench_inject1.json 2> $O/bench_inject1.err || { tail -20 $O/bench_inject1.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --workload config5 --steps 20 --warmup 5 --no-cpu > $O/bench_config5.json 2> $O/bench_config5.err || { tail -20 $O/bench_config5.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --workload config3 --steps 6 --warmup 2 --no-cpu > $O/bench_config3.json 2> $O/bench_config3.err || { tail -20 $O/bench_config3.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --workload config4 --steps 4 --warmup 2 --no-cpu > $O/bench_config4.json 2> $O/bench_config4.err || { tail -20 $O/bench_config4.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --workload config4 --multi-contexts 8 --steps 3 --inject 0.01 > $O/bench_config4_multi.json 2> $O/bench_config4_multi.err || { tail -20 $O/bench_config4_multi.err; exit 1; }
  for f in s48 inject1 config5 config3 config4; do python3 -c "import json;d=json.load(open('$O/bench_$f.json'));print('$f', d['value'], d['config']['level0'], d['config']['rlc_group'], d['roofline']['kernel'], d['roofline']['frac'])"; done
  python3 -c "import json;d=json.load(open('$O/bench_config4_multi.json'));print('config4_multi', d['value'], d['exact'], d['config'])"
  bash tools/gpu_pmc.sh 16 && cp -r gpurun_out/pmc $O/pmc
fi
