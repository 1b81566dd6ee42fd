#!/bin/bash
# Round-6 call S: as call R with sgb_digits back on the byte-stream block (k_sgb_sort 66 VGPRs); k_msm_bucket without the lambda (its additions had become a
# call per step with the accumulator through scratch) and with the ladder's
# base re-read from the output slot, the cofactor kernels' bases and rare-case
# operands re-read from their slots, the RLC / subgroup digits' SHA-256 block in
# registers, k_sgb_test's base re-read: the whole GPU suite, then the driver
# shape over four reps against HEAD before it (variants/pre_msm.so), then PMC.
#   bash tools/gpu_r06_r.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6s}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_tests.sh $D ${TESTS:-tests} || exit 1
for rep in 1 2 3 4; do
  for arm in product variants/pre_msm.so; do
    n=$(basename $arm .so)
    if [ $arm = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$arm; fi
    f=$O/${n}_s20_$rep.json
    timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 --steps 20 --warmup 5 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$f'));k=d['isolated_kernel_ms']
print('$n s20 $rep', d['value'], d['isolated_batch_ms']['total'], {x: k[x] for x in k if x in ('k_msm_bucket','k_sgb_sort')})"
  done
done
unset TBG_LIB
bash tools/gpu_pmc.sh 16 || exit 1
