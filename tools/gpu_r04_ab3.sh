#!/bin/bash
# Fallback-path A/B: 1 % invalid (20 / 5) and config 5 per build, fallback
# kernels' isolated times:  bash tools/gpu_r04_ab3.sh <outdir> <lib.so | product> ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4ab3}
shift
mkdir -p $O
cd $R
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$L; fi
  for a in "inj20 --steps 20 --warmup 5 --inject 0.01" "c5 --workload config5 --steps 20 --warmup 5"; do
    set -- $a
    tag=$1; shift
    f=$O/${n}_$tag.json
    timeout -k 10 300 python3 -u bench.py "$@" --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n $tag', d['value'], {x: k[x] for x in k if 'chunk' in x or 'cident' in x or 'sig_list' in x or 'verify_list' in x})"
  done
done
unset TBG_LIB
