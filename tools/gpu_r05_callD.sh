#!/bin/bash
# Round-5 call: the GPU suite with adaptive 8-duty Miller chunks, then an A/B
# against the chunk-4-only build: the driver shape (20/5) twice, 48 steps,
# and config 4's 125k-DV shard twice, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t4 || exit 1
O=$R/gpurun_out/r5c8
mkdir -p $O
run() {  # name lib out args...
  local n=$1 l=$2 f=$O/$3; shift 3
  if [ "$l" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$l; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 "$@" > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$3', d['value'], d['roofline']['frac'], d['ms_per_step'], {x: k[x] for x in k if 'miller' in x})"
}
for rep in 1 2; do
  run p product p_s20_$rep.json --steps 20 --warmup 5 || exit 1
  run c varlib/c4only.so c_s20_$rep.json --steps 20 --warmup 5 || exit 1
  run p product p_c4_$rep.json --workload config4 --steps 8 --warmup 2 || exit 1
  run c varlib/c4only.so c_c4_$rep.json --workload config4 --steps 8 --warmup 2 || exit 1
done
run p product p_s48.json --steps 48 --warmup 5 || exit 1
run c varlib/c4only.so c_s48.json --steps 48 --warmup 5 || exit 1
unset TBG_LIB
