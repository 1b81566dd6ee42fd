#!/bin/bash
# GPU suite at the working tree, then the 1 % invalid / config-5 A/B of the
# working build against varlib/prev.so (the build before the change):
#   bash tools/gpu_r04_merge.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4merge}
mkdir -p $O
cd $R
bash tools/gpu_r04_tests.sh ${1:-r4merge} || exit 1
for L in product varlib/prev.so; do
  n=$(basename $L .so)
  if [ "$L" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$L; fi
  for a in "inj20 --steps 20 --warmup 5 --inject 0.01" "inj48 --steps 48 --warmup 16 --inject 0.01" "c5 --workload config5 --steps 20 --warmup 5" "s20 --steps 20 --warmup 5"; do
    set -- $a
    tag=$1; shift
    f=$O/${n}_$tag.json
    timeout -k 10 300 python3 -u bench.py "$@" --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n $tag', d['value'], d.get('fallback_levels'), {x: k[x] for x in k if 'chunk' in x or 'cident' in x})"
  done
done
unset TBG_LIB
