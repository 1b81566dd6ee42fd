#!/bin/bash
# Round-5 A/B of builds / engine knobs on one box: an optional parity gate per
# variant library (the fixture suite + the config-2 oracle check through that
# library), then the driver's bench shape (20 / 5) and config 3 for every
# arm, interleaved (A B A B) so box drift hits both alike.
#   GATE=1 C3=1 bash tools/gpu_r05_ab.sh <outdir> <arm> ...
# arm = product | path/lib.so, optionally followed by @ and bench flags
# joined with commas: product@--subgroup-batch=2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ab}
shift
mkdir -p $O
cd $R
arm_lib() { echo "${1%%@*}"; }
arm_args() { [[ $1 == *@* ]] && echo "${1#*@}" | tr ',' ' '; }
arm_name() { local l=$(arm_lib $1); local a=$(arm_args $1 | tr -d ' -' | tr '=' '_'); echo "$(basename $l .so)${a:+_$a}"; }
libenv() { if [ "$1" = product ]; then unset TBG_LIB; else export TBG_LIB=$R/$1; fi; }
if [ "${GATE:-1}" = 1 ]; then
  for A in "$@"; do
    L=$(arm_lib $A)
    [ "$L" = product ] && continue
    n=$(basename $L .so)
    libenv $L
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_config2_full_batch_matches_oracle" \
      -m gpu -x -q -k "not native_library" --timeout 300 --timeout-method thread > $O/gate_$n.log 2>&1 || { tail -30 $O/gate_$n.log; exit 1; }
    tail -1 $O/gate_$n.log
  done
fi
for rep in 1 2; do
  for A in "$@"; do
    n=$(arm_name $A)
    libenv $(arm_lib $A)
    f=$O/${n}_s20_$rep.json
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --api-batches 0 --latency 0 $(arm_args $A) > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n s20 $rep', d['value'], d['roofline']['frac'], {x: k[x] for x in k if 'miller' in x or 'hash' in x})"
  done
done
if [ "${C3:-1}" = 1 ]; then
  for A in "$@"; do
    n=$(arm_name $A)
    libenv $(arm_lib $A)
    f=$O/${n}_c3.json
    timeout -k 10 300 python3 -u bench.py --workload config3 --steps 6 --warmup 2 --no-cpu --api-batches 0 --latency 0 $(arm_args $A) > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('$n c3', d['value'], {x: k[x] for x in k if 'miller' in x or 'hash' in x})"
  done
fi
unset TBG_LIB
