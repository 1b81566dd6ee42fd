#!/bin/bash
# Round-6 call Q: k_decode_sigs' inline root at window width 4
# (variants/dec_w4.so, 71 spilled VGPRs) vs width 3 (product, no spill):
# driver shape three reps, 48 steps once, interleaved.
#   bash tools/gpu_r06_q.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6q}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
for rep in 1 2 3 4; do
  for arm in product variants/dec_w4.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    if [ $rep = 4 ]; then args="--steps 48 --warmup 16"; tag=s48; else args="--steps 20 --warmup 5"; tag=s20_$rep; fi
    f=$O/${n}_${tag}.json
    timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$f'));k=d['isolated_kernel_ms']
print('$n $tag', d['value'], d['isolated_batch_ms']['total'], {x: k[x] for x in k if x in ('k_decode_sigs',)})"
  done
done
unset TBG_LIB
