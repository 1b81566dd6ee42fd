#!/bin/bash
# Width-4 exponentiation window A/B: driver shape twice and config 3 per build,
# with the decode / hash kernels' isolated times:
#   bash tools/gpu_r04_pow.sh <outdir> <lib.so | product> ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4pow}
shift
mkdir -p $O
cd $R
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$L; fi
  for a in "s20a --steps 20 --warmup 5" "s20b --steps 20 --warmup 5" "c3 --workload config3 --steps 6 --warmup 2"; do
    set -- $a
    tag=$1; shift
    f=$O/${n}_$tag.json
    timeout -k 10 300 python3 -u bench.py "$@" --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n $tag', d['value'], {x: k[x] for x in ('k_decode_sigs','k_hash_map','k_subgroup_sigs')})"
  done
done
unset TBG_LIB
