#!/bin/bash
# Round-5 call: parity / headline / config-2 oracle GPU tests with the
# two-point cofactor combination (k_hash_clear_fin), then A/B against the
# build before (fin0): driver shape twice and config 3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t12 "tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_fullsize.py::test_config2_full_batch_matches_oracle" || exit 1
GATE=0 C3=1 bash tools/gpu_r05_ab.sh r5fin product varlib/fin0.so
