#!/bin/bash
# A/B of library builds: driver shape (20 / 5) twice, 48 / 16 once, and the
# 1 % invalid line (20 / 5) once per build:
#   bash tools/gpu_r04_ab2.sh <outdir> <lib.so | product> ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4ab2}
shift
mkdir -p $O
cd $R
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$L; fi
  for rep in 1 2; do
    f=$O/${n}_s20_$rep.json
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));print('$n s20', d['value'], d['roofline']['frac'])"
  done
  f=$O/${n}_s48.json
  timeout -k 10 300 python3 -u bench.py --steps 48 --warmup 16 --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('$n s48', d['value'])"
  f=$O/${n}_inj.json
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --inject 0.01 --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('$n inject1', d['value'])"
done
unset TBG_LIB
