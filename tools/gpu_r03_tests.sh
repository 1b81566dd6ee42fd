#!/bin/bash
# The whole -m gpu suite in one process (progress lines per test in
# gpurun_out/<dir>/tests.log), bounded; stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r3tests}
mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -12
exit $rc
