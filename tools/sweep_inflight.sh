#!/bin/bash
# Parity tests, then the bench at several in-flight / HW-queue settings.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sweep
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for cfg in "8 16" "12 16" "16 16" "16 24" "24 32"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu --inflight $1 --hw-queues $2 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -5 $O/b_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$1_$2.json'));print('inflight',$1,'hwq',$2,d['value'],d['roofline']['frac'])"
done
