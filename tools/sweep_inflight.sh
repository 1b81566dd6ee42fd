#!/bin/bash
# Bench at several in-flight batch counts / HW-queue settings (no tests).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sweep
mkdir -p $O
cd $R
for cfg in "8 16" "12 16" "8 16" "12 16" "12 12"; do
  set -- $cfg
  if timeout -k 10 200 python bench.py --no-cpu --inflight $1 --hw-queues $2 > $O/b_$1_$2.json 2> $O/b_$1_$2.err; then
    python -c "import json;d=json.load(open('$O/b_$1_$2.json'));print('inflight',$1,'hwq',$2,d['value'])"
  else
    echo "inflight $1 hwq $2 failed: $(grep -o 'HSA_STATUS_ERROR[A-Z_]*\|EngineError.*' $O/b_$1_$2.err | head -2 | tr '\n' ' ')"; exit 0
  fi
done
