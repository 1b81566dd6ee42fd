#!/bin/bash
# Round-3 record at HEAD.  part A: the -m gpu suite, then the driver's bench
# command under a rocprofv3 kernel trace (+ the roofline recomputed from it).
# part B: the side lines (48 steps, 1 % invalid, configs 5 / 3 / 4) and the
# PMC traffic passes.        bash tools/gpu_r03_final.sh <A|B> <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=${2:-r3final}
cd $R
if [ "$1" = A ]; then
  bash tools/gpu_r03_tests.sh $O/tests && bash tools/gpu_r03_bench.sh $O/headline headline
else
  mkdir -p gpurun_out/$O/side
  S=gpurun_out/$O/side
  timeout -k 10 300 python3 -u bench.py --steps 48 --warmup 16 --no-cpu --api-batches 0 > $S/bench_s48.json 2> $S/bench_s48.err || { tail -20 $S/bench_s48.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --inject 0.01 --no-cpu --api-batches 0 > $S/bench_inject1.json 2> $S/bench_inject1.err || { tail -20 $S/bench_inject1.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --steps 48 --warmup 16 --inject 0.01 --no-cpu --api-batches 0 > $S/bench_inject1_s48.json 2> $S/bench_inject1_s48.err || { tail -20 $S/bench_inject1_s48.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --workload config5 --steps 20 --warmup 5 --no-cpu > $S/bench_config5.json 2> $S/bench_config5.err || { tail -20 $S/bench_config5.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --workload config3 --steps 6 --warmup 2 --cpu-seconds 10 > $S/bench_config3.json 2> $S/bench_config3.err || { tail -20 $S/bench_config3.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --workload config4 --steps 4 --warmup 2 --no-cpu > $S/bench_config4.json 2> $S/bench_config4.err || { tail -20 $S/bench_config4.err; exit 1; }
  for f in s48 inject1 inject1_s48 config5 config3 config4; do python3 -c "import json;d=json.load(open('$S/bench_$f.json'));print('$f', d['value'], d['config']['level0'], d['config']['rlc_group'], d['roofline']['kernel'], d['roofline']['frac'])"; done
  bash tools/gpu_pmc.sh 16 && cp -r gpurun_out/pmc gpurun_out/$O/pmc
fi
