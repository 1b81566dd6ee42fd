#!/bin/bash
# Invalid-path A/B: 1 % invalid partials (20 / 5) and config 5 (mixed
# injections) per library build: bash tools/gpu_r04_inv.sh <outdir> <lib.so | product> ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4inv}
shift
mkdir -p $O
cd $R
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$L; fi
  timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --inject 0.01 --no-cpu --api-batches 0 > $O/${n}_inject1.json 2> $O/${n}_inject1.err || { tail -20 $O/${n}_inject1.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --workload config5 --steps 20 --warmup 5 --no-cpu --api-batches 0 > $O/${n}_config5.json 2> $O/${n}_config5.err || { tail -20 $O/${n}_config5.err; exit 1; }
  for f in inject1 config5; do
    python3 -c "import json;d=json.load(open('$O/${n}_$f.json'));print('$n $f', d['value'], d['ms_per_step'], sorted(d['isolated_kernel_ms'].items(), key=lambda kv: -kv[1])[:8])"
  done
done
unset TBG_LIB
