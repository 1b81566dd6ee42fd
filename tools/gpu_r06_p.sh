#!/bin/bash
# Round-6 call P: the aggregation list kernels on capped looping grids: the
# whole GPU suite, then 1 % invalid / config 5 / driver shape A/B against
# HEAD before it (variants/pre_agg.so), interleaved, two reps.
#   bash tools/gpu_r06_p.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6p}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_tests.sh $D ${TESTS:-tests} || exit 1
for rep in 1 2; do
  for wl in "inj1:--steps 20 --warmup 5 --inject 0.01" "c5:--workload config5 --steps 20 --warmup 5" "s20:--steps 20 --warmup 5"; do
    tag=${wl%%:*}; args=${wl#*:}
    for arm in product variants/pre_agg.so; do
      n=$(basename $arm .so)
      if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
      f=$O/${n}_${tag}_$rep.json
      timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "
import json;d=json.load(open('$f'));k=d['isolated_kernel_ms']
print('$n $tag $rep', d['value'], d['isolated_batch_ms']['aggregate'], {x: k[x] for x in k if 'aggregate' in x})"
    done
  done
done
unset TBG_LIB
