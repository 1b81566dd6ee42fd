#!/bin/bash
# Round-5 call: shape / headline / parity / replay GPU tests with the
# SIMD-unit shape model and replay-plan reshaping, then A/B against the
# build that keeps the submitted shapes in replays (rs0): driver shape
# twice, 48 steps, config 4, config 3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t9 "tests/test_gpu_shape.py tests/test_gpu_headline.py tests/test_gpu_parity.py $(ls tests/test_gpu_replay*.py 2>/dev/null)" || exit 1
O=$R/gpurun_out/r5rs
mkdir -p $O
run() {  # lib name args...
  local l=$1 n=$2 f=$O/$2.json; shift 2
  if [ "$l" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$l; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 "$@" > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n', d['value'], d['ms_per_step'], d['config'].get('rlc_chunk'), k.get('k_miller_hex<MILLER_L0>'), d['kernel_ms_per_step'].get('verify'))"
}
for rep in 1 2; do
  run product p_s20_$rep --steps 20 --warmup 5 || exit 1
  run varlib/rs0.so c_s20_$rep --steps 20 --warmup 5 || exit 1
done
run product p_s48 --steps 48 --warmup 5 || exit 1
run varlib/rs0.so c_s48 --steps 48 --warmup 5 || exit 1
run product p_c4 --workload config4 --steps 8 --warmup 2 || exit 1
run product p_c3 --workload config3 --steps 6 --warmup 2 || exit 1
unset TBG_LIB
