#!/bin/bash
# A/B of library builds on the driver's bench shape (20 / 5) and the 48-step
# line: bash tools/gpu_r04_ab.sh <outdir> <lib.so | product> ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4ab}
shift
mkdir -p $O
cd $R
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$L; fi
  for rep in 1 2; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 > $O/${n}_s20_$rep.json 2> $O/${n}_s20_$rep.err || { tail -20 $O/${n}_s20_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${n}_s20_$rep.json'));print('$n s20', d['value'], d['roofline']['frac'], {k: v for k, v in d['isolated_kernel_ms'].items() if k in ('k_l0_final','k_msm_bucket','k_msm_sum','k_msm_tree','k_msm_tree_final','k_l0_lines','k_l0_tree')})"
  done
  timeout -k 10 300 python3 -u bench.py --steps 48 --warmup 16 --no-cpu --api-batches 0 > $O/${n}_s48.json 2> $O/${n}_s48.err || { tail -20 $O/${n}_s48.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${n}_s48.json'));print('$n s48', d['value'])"
done
unset TBG_LIB
