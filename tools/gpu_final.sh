#!/bin/bash
# End-of-round evidence in one call: C-ABI thread tests + the whole -m gpu
# suite, the round bench (default line with CPU baseline, driver-style 20/5,
# rocprof kernel stats), PMC traffic, 1 %-invalid and config-4 side lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh && bash tools/gpu_bench_round.sh && bash tools/gpu_evidence.sh
