#!/bin/bash
# The driver's own command, twice, without a profiler: bash tools/gpu_r04_driver.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4drv}
mkdir -p $O
cd $R
for rep in 1 2; do
  f=$O/driver_$rep.json
  timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('driver', $rep, d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
done
