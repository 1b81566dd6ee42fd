#!/bin/bash
# Round-5 call: the GPU suite with the 8-entry per-key window tables
# (TBG_PK_W2), then A/B against the pair tables (pk2): driver shape twice,
# config 3, 1 % invalid.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t10 || exit 1
O=$R/gpurun_out/r5pk
mkdir -p $O
run() {  # lib name args...
  local l=$1 n=$2 f=$O/$2.json; shift 2
  if [ "$l" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$l; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 "$@" > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n', d['value'], d['ms_per_step'], k.get('k_rlc_g1_l0'), k.get('k_rlc_partial2'))"
}
for rep in 1 2; do
  run product p_s20_$rep --steps 20 --warmup 5 || exit 1
  run varlib/pk2.so c_s20_$rep --steps 20 --warmup 5 || exit 1
done
run product p_c3 --workload config3 --steps 6 --warmup 2 || exit 1
run varlib/pk2.so c_c3 --workload config3 --steps 6 --warmup 2 || exit 1
run product p_inj --steps 20 --warmup 5 --inject 0.01 || exit 1
run varlib/pk2.so c_inj --steps 20 --warmup 5 --inject 0.01 || exit 1
unset TBG_LIB
