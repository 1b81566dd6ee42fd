#!/bin/bash
# Round-6 call E: group MSM with LDS-aggregated bucket ordering: the RLC
# GPU tests, then 1 % invalid, config 5 and the clean driver shape, A/B
# against the per-partial build (variants/gm0.so), interleaved.
#   bash tools/gpu_r06_e.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6e}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_tests.sh $D ${TESTS:-tests} || exit 1
for rep in 1 2; do
  for arm in product variants/gm0.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    for wl in "inj1:--inject 0.01" "c5:--workload config5" "clean:"; do
      tag=${wl%%:*}; args=${wl#*:}
      f=$O/${n}_${tag}_$rep.json
      timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n $tag $rep', d['value'], d['isolated_batch_ms']['combine'], d['isolated_batch_ms']['total'], {x: k[x] for x in k if 'gm' in x or 'partial2' in x or 'rlc_g1' in x or 'duty_sum' in x})"
    done
  done
done
unset TBG_LIB
