#!/bin/bash
# GPU test pass (run on the box through gpurun): the C-ABI thread test (plain
# and ASan-on-host builds, when built) and the whole -m gpu suite in one
# process, each bounded; logs under gpurun_out/tests/.  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/tests
mkdir -p $O
cd $R
if [ -x tests/cabi/cabi_threads ]; then
  timeout -k 10 120 tests/cabi/cabi_threads > $O/cabi_threads.log 2>&1 || { echo "cabi_threads rc=$?"; tail -20 $O/cabi_threads.log; exit 1; }
  tail -1 $O/cabi_threads.log
fi
if [ -x tests/cabi/cabi_threads_asan ]; then
  ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0 timeout -k 10 180 tests/cabi/cabi_threads_asan > $O/cabi_threads_asan.log 2>&1 || { echo "cabi_threads_asan rc=$?"; tail -30 $O/cabi_threads_asan.log; exit 1; }
  tail -1 $O/cabi_threads_asan.log
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${@} > $O/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/gpu_tests.log | tail -40
exit $rc
