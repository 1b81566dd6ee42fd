#!/bin/bash
# Round-5 call: the GPU suite with the level-0 launch shape rule (l0_shape),
# an A/B against the (16, 4)-only build on config 4's shard, 48 and 20
# steps, then the 1 % invalid workload and config 5 under the three level-1g
# routings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t5 || exit 1
O=$R/gpurun_out/r5shape
mkdir -p $O
run() {  # lib out args...
  local l=$1 n=$2 f=$O/$2.json; shift 2
  if [ "$l" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$l; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 "$@" > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];r=d['roofline'];print('$n', d['value'], r['frac'], r['kernel'], d['ms_per_step'], d['config'].get('rlc_chunk'), {x: k[x] for x in k if 'miller' in x})"
}
for rep in 1 2; do
  run product p_c4_$rep --workload config4 --steps 8 --warmup 2 || exit 1
  run varlib/c4only.so c_c4_$rep --workload config4 --steps 8 --warmup 2 || exit 1
done
run product p_s48 --steps 48 --warmup 5 || exit 1
run varlib/c4only.so c_s48 --steps 48 --warmup 5 || exit 1
run product p_s20 --steps 20 --warmup 5 || exit 1
for g in 0 1 2; do
  run product inj_g$g --steps 20 --warmup 5 --inject 0.01 --gident $g || exit 1
done
for g in 0 2; do
  run product c5_g$g --workload config5 --steps 20 --warmup 5 --gident $g || exit 1
done
unset TBG_LIB
