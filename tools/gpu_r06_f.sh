#!/bin/bash
# Round-6 call F: level-0 shapes with one-chunk groups of 5..16 duties
# (VERDICT r05 item 7): the shape / replay / level-0 GPU tests, then the
# driver shape (20 / 5), 48 steps, config 4's shard and config 3, A/B
# against the old candidate set (variants/shape0.so), interleaved.
#   bash tools/gpu_r06_f.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6f}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_tests.sh $D ${TESTS:-"tests/test_gpu_shape.py tests/test_gpu_replay_shape.py tests/test_gpu_headline.py tests/test_gpu_parity.py"} || exit 1
for rep in 1 2; do
  for arm in product variants/shape0.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    for wl in "s20:--steps 20 --warmup 5" "c4:--workload config4 --steps 20 --warmup 5" "s48:--steps 48 --warmup 16" "c3:--workload config3 --steps 20 --warmup 5"; do
      tag=${wl%%:*}; args=${wl#*:}
      [ $rep = 2 ] && [ $tag = c3 ] && continue
      f=$O/${n}_${tag}_$rep.json
      timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n $tag $rep', d['value'], d['config']['rlc_group'], d['config']['rlc_chunk'], d['roofline']['frac'], {x: k[x] for x in k if 'miller' in x or 'l0_' in x})"
    done
  done
done
unset TBG_LIB
