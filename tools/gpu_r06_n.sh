#!/bin/bash
# Round-6 call N: the driver shape, four reps interleaved over HEAD, HEAD
# with the complete additions inline in k_msm_bucket (variants/msmx0.so),
# HEAD with the width-3 SSWU window (variants/sswu_w3.so) and the evidence
# build before the scratch work (variants/hash_old.so); one 48-step run each.
#   bash tools/gpu_r06_n.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6n}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
for rep in 1 2 3 4 5; do
  for arm in product variants/msmx0.so variants/sswu_w3.so variants/hash_old.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    if [ $rep = 5 ]; then args="--steps 48 --warmup 16"; tag=s48; else args="--steps 20 --warmup 5"; tag=s20_$rep; fi
    f=$O/${n}_${tag}.json
    timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$f'));k=d['isolated_kernel_ms']
print('$n $tag', d['value'], d['isolated_batch_ms']['total'], {x: k[x] for x in k if x in ('k_hash_sswu','k_hash_map','k_msm_bucket')})"
  done
done
unset TBG_LIB
