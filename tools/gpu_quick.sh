#!/bin/bash
# Parity tests + one default bench line (no CPU leg); stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/quick
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac'],d['isolated_batch_ms'])"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu --steps 4 --inflight 1 > $O/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu --steps 4 --inflight 1 > $O/pmc_fetch.log 2>&1
cd $R && python tools/pmc_traffic.py $O $O/traffic.json
