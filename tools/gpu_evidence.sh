#!/bin/bash
# Round evidence for the current build: PMC traffic passes (tools/gpu_pmc.sh),
# the 1 %-invalid side measurement and the config-4 shard bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/evidence
mkdir -p $O
cd $R
bash tools/gpu_pmc.sh 16 > $O/pmc.txt 2>&1 || { tail -20 $O/pmc.txt; exit 1; }
tail -12 $O/pmc.txt
timeout -k 10 300 python bench.py --no-cpu --api-batches 0 --inject 0.01 > $O/inject1.json 2> $O/inject1.err || { tail -5 $O/inject1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/inject1.json'));print('inject 1%', d['value'], d['config']['rlc_group'], d['config']['level0'])"
timeout -k 10 300 python bench.py --no-cpu --api-batches 0 --workload config4 --steps 6 --warmup 2 > $O/config4.json 2> $O/config4.err || { tail -5 $O/config4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/config4.json'));print('config4', d['value'], d['ms_per_step'], d['config']['level0'])"
