#!/bin/bash
# Round-6 call B: the batched subgroup test's adaptive group size (VERDICT
# r05 item 3): its GPU tests, then config 5 and the headline at 20 steps.
#   bash tools/gpu_r06_b.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6b}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
bash tools/gpu_tests.sh $D "tests/test_gpu_sgb.py tests/test_gpu_fullsize.py::test_config5_mixed_injections_match_oracle" || exit 1
timeout -k 10 600 python3 -u bench.py --workload config5 --steps 20 --warmup 5 --no-cpu --latency 0 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5.json'));k=d['isolated_kernel_ms'];print('c5', d['value'], d['subgroup_batch'], d['isolated_batch_ms'], {x: k[x] for x in k if 'sgb' in x or 'subgroup' in x or 'decode' in x})"
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --latency 0 > $O/s20.json 2> $O/s20.err || { tail -20 $O/s20.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/s20.json'));print('s20', d['value'], d['roofline']['frac'], d['subgroup_batch'])"
