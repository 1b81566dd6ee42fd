#!/bin/bash
# Round-5 call: batched-subgroup / parity / headline GPU tests with the
# folded bucket slices (k_sgb_fold), then A/B against the 30-addition
# running sums (sgb30) on the driver shape and config 3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t8 "tests/test_gpu_sgb.py tests/test_gpu_parity.py tests/test_gpu_headline.py" || exit 1
GATE=0 C3=1 bash tools/gpu_r05_ab.sh r5fold product varlib/sgb30.so
