#!/bin/bash
# Round-6 evidence at HEAD, part A: smoke(), the driver's bench command under
# a rocprofv3 kernel trace (+ the roofline recomputed from that trace and the
# timed region's timeline), then the same command without the profiler.
#   bash tools/gpu_r06_final.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6final}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20w5.json 2> $O/bench_s20w5.err || { tail -20 $O/bench_s20w5.err; exit 1; }
cd $R && python3 tools/roofline_from_trace.py $O/prof/run_kernel_trace.csv $O/bench_s20w5.json --out $O/roofline_check.json || exit 1
python3 tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt 2>&1 || true
python3 -c "import json;d=json.load(open('$O/bench_s20w5.json'));r=d['roofline'];print('s20 rocprof', d['value'], r['kernel'], r['frac'], r.get('frac_fp300'), d['api_pipeline']['value'] if d['api_pipeline'] else None, d['cpu_baseline'], json.dumps(d.get('small_batch_latency')))"
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || { tail -20 $O/driver.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver.json'));r=d['roofline'];print('driver', d['value'], r['frac'], d['api_pipeline']['value'])"
