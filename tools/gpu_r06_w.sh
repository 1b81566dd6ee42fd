#!/bin/bash
# Round-6 call W: the AMDGPU machine scheduler's ILP strategies for the whole
# library (variants/ilp.so: -mllvm -amdgpu-sched-strategy=max-ilp;
# variants/itilp.so: =iterative-ilp) vs the product (default strategy):
# the driver shape, arms interleaved, with every big kernel's isolated time.
#   bash tools/gpu_r06_w.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6w}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
for rep in ${REPS:-1 2}; do
  for arm in ${ARMS:-product ilp itilp}; do
    [ $arm = product ] || [ -f variants/$arm.so ] || continue
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/variants/$arm.so; fi
    f=$O/${arm}_s20_$rep.json
    timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 --steps 20 --warmup 5 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$f'));k=d['isolated_kernel_ms']
print('$arm $rep', d['value'], [x['exact'] for x in d['ranks_exact_after_clock']], {n[:16]: round(k[n], 2) for n in list(k)[:10]})"
    unset TBG_LIB
  done
done
