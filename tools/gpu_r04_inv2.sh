#!/bin/bash
# Clean (20 / 5 x2, 48 / 16), 1 % invalid (20 / 5) and config 5 per library
# build: bash tools/gpu_r04_inv2.sh <outdir> <lib.so | product> ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4ab}
shift
mkdir -p $O
cd $R
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$L; fi
  for run in "s20_1 --steps 20 --warmup 5" "s20_2 --steps 20 --warmup 5" "s48 --steps 48 --warmup 16" \
             "inject1 --steps 20 --warmup 5 --inject 0.01" "config5 --workload config5 --steps 20 --warmup 5"; do
    set -- $run
    tag=$1; shift
    timeout -k 10 400 python3 -u bench.py --no-cpu --api-batches 0 "$@" > $O/${n}_$tag.json 2> $O/${n}_$tag.err || { tail -20 $O/${n}_$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${n}_$tag.json'));k=d['isolated_kernel_ms'];print('$n $tag', d['value'], d['roofline']['frac'], {x: k.get(x) for x in ('k_l0_inv','k_rlc_duty_sum<DSUM_L0_P>','k_aggregate<true>','k_rlc_group_final','k_rlc_check_chunks','k_hash_map') if k.get(x)})"
  done
done
unset TBG_LIB
