#!/bin/bash
# Round-5 A/B on invalid traffic: 1 % injected wrong-message partials and
# config 5 (mixed duties, every invalid kind), driver step counts (20 / 5),
# arms interleaved (A B A B), fallback kernels' isolated times printed.
#   bash tools/gpu_r05_inv.sh <outdir> <arm> ...   (arms as in gpu_r05_ab.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5inv}
shift
mkdir -p $O
cd $R
arm_lib() { echo "${1%%@*}"; }
arm_args() { [[ $1 == *@* ]] && echo "${1#*@}" | tr ',' ' '; }
arm_name() { local l=$(arm_lib $1); local a=$(arm_args $1 | tr -d ' -' | tr '=' '_'); echo "$(basename $l .so)${a:+_$a}"; }
libenv() { if [ "$1" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$1; fi; }
ARMS=("$@")
for rep in ${REPS:-1 2}; do
  for A in "${ARMS[@]}"; do
    n=$(arm_name $A)
    libenv $(arm_lib $A)
    for w in "inj --inject 0.01" "c5 --workload config5"; do
      tag=${w%% *}
      f=$O/${n}_${tag}_$rep.json
      timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 --latency 0 ${w#* } $(arm_args $A) > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n $tag $rep', d['value'], d['config']['level0'], d['config']['rlc_group'], d.get('subgroup_batch'), {x: k[x] for x in list(k)[:6]})"
    done
  done
done
unset TBG_LIB
