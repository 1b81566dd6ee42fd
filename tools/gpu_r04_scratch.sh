#!/bin/bash
# Scratch-limit probe: the same benches under the HSA runtime's default
# scratch handling and with its per-dispatch limit raised / thread limiter off.
#   bash tools/gpu_r04_scratch.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4scr}
mkdir -p $O
cd $R
run() {  # tag, env..., then bench args after --
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  f=$O/$tag.json
  env "${envs[@]}" timeout -k 10 300 python3 -u bench.py "$@" --no-cpu --api-batches 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$tag', d['value'], {x: k[x] for x in sorted(k, key=lambda y: -k[y])[:12]})"
}
for cfg in "def" "lim HSA_SCRATCH_SINGLE_LIMIT=8589934592" "nolim HSA_NO_SCRATCH_THREAD_LIMITER=1"; do
  set -- $cfg
  tag=$1; shift
  run ${tag}_inj20 "$@" -- --steps 20 --warmup 5 --inject 0.01 || exit 1
  run ${tag}_s20 "$@" -- --steps 20 --warmup 5 || exit 1
done
