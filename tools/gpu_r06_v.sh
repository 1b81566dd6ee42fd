#!/bin/bash
# Round-6 call V: the run's level-0 Miller kernels joined behind every
# launch's signature side (variants/join.so, -DTBG_L0_JOIN=1) vs the product;
# the driver shape REPS times per arm, arms interleaved (the first arm
# alternating), then 48 steps once each.
#   bash tools/gpu_r06_v.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6v}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
run() {  # arm tag args...
  local arm=$1 tag=$2; shift 2
  if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/variants/$arm.so; fi
  local f=$O/${arm}_${tag}.json
  timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 "$@" > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$f'));k=d['kernel_ms_per_step']
print('$arm $tag', d['value'], d['ms_per_step'], k['combine'], k['verify'], [x['exact'] for x in d['ranks_exact_after_clock']])"
  unset TBG_LIB
}
for rep in ${REPS:-1 2 3 4 5 6 7}; do
  if [ $((rep % 2)) = 1 ]; then arms="product join"; else arms="join product"; fi
  for arm in $arms; do run $arm s20_$rep --steps 20 --warmup 5 || exit 1; done
done
for arm in product join; do run $arm s48 --steps 48 --warmup 16 || exit 1; done
