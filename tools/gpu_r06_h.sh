#!/bin/bash
# Round-6 call H: fallback passes sized by the expected list length (grid-
# stride pass kernels): the whole GPU suite, the limb microbench, then the
# driver shape, 48 steps and 1 % invalid A/B against every-pass-full
# (variants/fbx0.so), interleaved.
#   bash tools/gpu_r06_h.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6h}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_tests.sh $D ${TESTS:-tests} || exit 1
timeout -k 10 120 tools/microbench/limb_ab > $O/limb_ab.txt 2>&1 || { tail -5 $O/limb_ab.txt; exit 1; }
python3 tools/microbench/limb_ab_check.py $O/limb_ab.txt && cat $O/limb_ab.txt | grep waves
for rep in 1 2; do
  for arm in product variants/fbx0.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    for wl in "s20:--steps 20 --warmup 5" "inj1:--steps 20 --warmup 5 --inject 0.01" "s48:--steps 48 --warmup 16"; do
      tag=${wl%%:*}; args=${wl#*:}
      [ $rep = 2 ] && [ $tag = s48 ] && continue
      f=$O/${n}_${tag}_$rep.json
      timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json;d=json.load(open('$f'));print('$n $tag $rep', d['value'], d['roofline']['frac'], d['isolated_batch_ms']['total'])"
    done
  done
done
unset TBG_LIB
