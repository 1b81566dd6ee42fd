#!/bin/bash
# Round-3 check: the new headline-shape / config-3 / C-ABI tests and the DKG
# tests, then the driver's bench command under a rocprofv3 kernel trace, and
# the roofline recomputed from that trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_dkg.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd $R && python3 tools/roofline_from_trace.py $O/prof/run_kernel_trace.csv $O/bench.json --out $O/roofline_check.json
