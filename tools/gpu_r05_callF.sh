#!/bin/bash
# Round-5 call: the GPU suite with interleaved square roots (two SSWU maps /
# two signatures per lane), then A/B: product vs one signature per lane
# (dx1) vs the build before both (c4only: also (16, 4)-only shapes), on the
# driver shape (20 / 5, twice) and config 3 -- isolated k_hash_map and
# k_decode_sigs times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t6 || exit 1
C3=1 GATE=0 bash tools/gpu_r05_ab.sh r5sqrt product varlib/dx1.so varlib/c4only.so
