#!/bin/bash
# Decode-bound A/B: config 3 (7-of-10, 100k DVs) and the 20 / 5 headline per
# library build: bash tools/gpu_r04_c3.sh <outdir> <lib.so | product> ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4c3}
shift
mkdir -p $O
cd $R
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$L; fi
  timeout -k 10 400 python3 -u bench.py --workload config3 --steps 6 --warmup 2 --no-cpu --api-batches 0 > $O/${n}_config3.json 2> $O/${n}_config3.err || { tail -20 $O/${n}_config3.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 > $O/${n}_s20.json 2> $O/${n}_s20.err || { tail -20 $O/${n}_s20.err; exit 1; }
  for f in config3 s20; do
    python3 -c "import json;d=json.load(open('$O/${n}_$f.json'));k=d['isolated_kernel_ms'];print('$n $f', d['value'], {x: k.get(x) for x in ('k_decode_sigs','k_subgroup_sigs','k_miller_hex<MILLER_L0>')})"
  done
done
unset TBG_LIB
