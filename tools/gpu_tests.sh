#!/bin/bash
# The -m gpu suite (or the tests named in $2) in one process, progress per
# test in gpurun_out/<dir>/tests.log; bounded; stops at the first failure.
#   bash tools/gpu_tests.sh <outdir> [pytest selection]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4tests}
SEL=${2:-tests}
mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest $SEL -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|slowest|s call" $O/tests.log | tail -30
exit $rc
