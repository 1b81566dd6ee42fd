#!/bin/bash
# Round-6 call L: + the Miller line steps in a liveness order with early
# stores (k_lines_h without spills): the whole GPU suite, then driver shape /
# 1 % invalid / 48 steps A/B against HEAD (variants/hash_old.so) and the
# width-4 SSWU window (variants/sswu_w4.so), interleaved; PMC traffic last.
#   bash tools/gpu_r06_l.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6l}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_tests.sh $D ${TESTS:-tests} || exit 1
for rep in 1 2; do
  for arm in product variants/hash_old.so variants/sswu_w4.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    for wl in "s20:--steps 20 --warmup 5" "inj1:--steps 20 --warmup 5 --inject 0.01" "s48:--steps 48 --warmup 16"; do
      tag=${wl%%:*}; args=${wl#*:}
      [ $rep = 2 ] && [ $tag = s48 ] && continue
      f=$O/${n}_${tag}_$rep.json
      timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "
import json;d=json.load(open('$f'));k=d['isolated_kernel_ms']
print('$n $tag $rep', d['value'], d['isolated_batch_ms'], {x: k[x] for x in k if x in ('k_hash_sswu','k_hash_map','k_lines_h','k_decode_sigs')})"
    done
  done
done
unset TBG_LIB
bash tools/gpu_pmc.sh 16 || exit 1
