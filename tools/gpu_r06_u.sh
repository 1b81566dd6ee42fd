#!/bin/bash
# Round-6 call U: the 20-step run as one launch of 20 caller batches
# (--inflight 1 --merge 20) and as 10 + 10 (--inflight 2) vs the default
# 7 + 7 + 6 over three slots; interleaved, two reps.
#   bash tools/gpu_r06_u.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6u}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
for rep in ${REPS:-1 2}; do
  for arm in ${ARMS:-default one two}; do
    case $arm in
      default) extra="" ;;
      one) extra="--inflight 1 --merge 20" ;;
      two) extra="--inflight 2" ;;
    esac
    f=$O/${arm}_s20_$rep.json
    timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 --steps 20 --warmup 5 $extra > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$f'))
print('$arm $rep', d['value'], d['ms_per_step'], [x['exact'] for x in d['ranks_exact_after_clock']])"
  done
done
