#!/bin/bash
# Round-6 call M: HEAD after the scratch work (width-4 SSWU window, the
# level-0 bucket kernel's rare case out of line): the whole GPU suite, then
# A/B against the round-6 evidence build (variants/hash_old.so) on the
# driver shape (twice), 48 steps, 1 % invalid and config 5, interleaved.
#   bash tools/gpu_r06_m.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6m}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_tests.sh $D ${TESTS:-tests} || exit 1
for wl in "s20:--steps 20 --warmup 5" "s48:--steps 48 --warmup 16" "inj1:--steps 20 --warmup 5 --inject 0.01" "c5:--workload config5 --steps 20 --warmup 5" "s20b:--steps 20 --warmup 5"; do
  tag=${wl%%:*}; args=${wl#*:}
  for arm in product variants/hash_old.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    f=$O/${n}_${tag}.json
    timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$f'));k=d['isolated_kernel_ms']
print('$n $tag', d['value'], d['isolated_batch_ms']['total'], {x: k[x] for x in k if x in ('k_hash_sswu','k_hash_map','k_lines_h','k_decode_sigs','k_msm_bucket')})"
  done
done
unset TBG_LIB
