#!/bin/bash
# Round-6 call A: the driver's 1-GPU bench command (engine on its own HIP
# runtime, no torch in the process), the --gpus 2 self-launch on the one GPU
# (both ranks on device 0), then the GPU suite.
#   bash tools/gpu_r06_a.sh <outdir>
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${1:-r6a}
O=$R/gpurun_out/$D
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err || { tail -20 $O/n1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/n1.json'));print('n1', d['value'], d['roofline']['frac'], d['api_pipeline']['value'], d['ranks_exact_after_clock'])"
timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/n2.json'));print('n2', d['n_gpus'], d['value'], d['ms_per_step'], d['ranks_exact_after_clock'])"
grep -h amdhip /proc/self/maps > /dev/null 2>&1
bash tools/gpu_tests.sh $D || exit 1
