#!/bin/bash
# One GPU measurement pass (run on the box through gpurun): parity tests,
# the bench line (with the CPU baseline), a rocprofv3 kernel-trace summary of
# the same bench, and the two PMC traffic passes (FETCH_SIZE / WRITE_SIZE in
# separate runs, as MI355X_MICROARCH.md prescribes).  Every step is bounded
# and the script stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round
mkdir -p $O
cd $R
echo "== tests"; timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
echo "== bench"; timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp
echo "== rocprof stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu > $O/bench_prof.json 2> $O/prof.log || { tail -20 $O/prof.log; exit 1; }
echo "== pmc fetch"; timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu --steps 4 --inflight 1 > $O/pmc_fetch.log 2>&1
echo "== pmc write"; timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu --steps 4 --inflight 1 > $O/pmc_write.log 2>&1
echo "== done"
