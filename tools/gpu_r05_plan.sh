#!/bin/bash
# Round-5 call: the driver's 20-step command under different replay plans
# (how the 20 caller batches are grouped into launches / slots in flight).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r5plan
mkdir -p $O
run() {  # name args...
  local n=$1 f=$O/$1.json; shift
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 --latency 0 "$@" > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('$n', d['value'], d['ms_per_step'])"
}
run def1 || exit 1
run s8_7_5 --split 8,7,5 || exit 1
run s10_6_4 --split 10,6,4 || exit 1
run s12_8 --split 12,8 || exit 1
run s10_10 --split 10,10 || exit 1
run s16_4 --split 16,4 || exit 1
run inf4 --inflight 4 || exit 1
run inf2 --inflight 2 || exit 1
run def2 || exit 1
