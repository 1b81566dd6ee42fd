#!/bin/bash
# Round-5 call: parity / headline / config-2 oracle GPU tests with Q0 + Q1
# moved from k_hash_map into k_hash_clear_x1, then A/B against the build
# before (hadd): driver shape twice and config 3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t11 "tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_fullsize.py::test_config2_full_batch_matches_oracle" || exit 1
GATE=0 C3=1 bash tools/gpu_r05_ab.sh r5hadd product varlib/hadd.so
