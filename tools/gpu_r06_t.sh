#!/bin/bash
# Round-6 call T: odd slots running the per-signature chain first
# (variants/alt.so, -DTBG_ALT_ORDER=1) vs the product (every slot: the
# per-message chain first): driver shape three reps, 48 steps once, 1 %
# invalid once, interleaved.
#   bash tools/gpu_r06_t.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6t}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
for rep in 1 2 3 4 5; do
  for arm in product variants/alt.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    case $rep in
      4) args="--steps 48 --warmup 16"; tag=s48 ;;
      5) args="--steps 20 --warmup 5 --inject 0.01"; tag=inv1 ;;
      *) args="--steps 20 --warmup 5"; tag=s20_$rep ;;
    esac
    f=$O/${n}_${tag}.json
    timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$f'))
print('$n $tag', d['value'], d['ms_per_step'], d.get('exact_after_clock', d.get('ranks_exact_after_clock')))"
  done
done
unset TBG_LIB
