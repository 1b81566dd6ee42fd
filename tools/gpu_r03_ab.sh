#!/bin/bash
# Parity subset (level-0 shapes) then a bench A/B of an environment knob:
#   bash tools/gpu_r03_ab.sh <outdir> <tests-k-expr or -> VAR=a VAR=b ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3ab}
K=$2
shift 2
mkdir -p $O
cd $R
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -25
  [ $rc -eq 0 ] || exit $rc
fi
for kv in "$@"; do
  n=$(echo "$kv" | tr '/=' '__')
  timeout -k 10 300 env $kv python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$n.json'));r=d['roofline'];print('$kv', d['value'], d['config']['level0'], r['kernel'], r['frac'], r['launch_ms'], d['isolated_batch_ms']['verify'])"
done
