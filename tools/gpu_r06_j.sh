#!/bin/bash
# Round-6 call J: the split hash_to_G2 map (k_hash_map + k_hash_sswu, VERDICT
# r05 item 6): the whole GPU suite, then the driver shape and 1 % invalid A/B
# against the one-kernel map (variants/hash_old.so, HEAD's sources), with the
# isolated per-kernel times of the hash stage.
#   bash tools/gpu_r06_j.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6j}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_tests.sh $D ${TESTS:-tests} || exit 1
for rep in 1 2; do
  for arm in product variants/hash_old.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    for wl in "s20:--steps 20 --warmup 5" "inj1:--steps 20 --warmup 5 --inject 0.01"; do
      tag=${wl%%:*}; args=${wl#*:}
      f=$O/${n}_${tag}_$rep.json
      timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "
import json;d=json.load(open('$f'));k=d['isolated_kernel_ms']
print('$n $tag $rep', d['value'], d['isolated_batch_ms']['hash'], {x: k[x] for x in k if 'hash' in x})"
    done
  done
done
unset TBG_LIB
