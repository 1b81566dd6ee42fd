#!/bin/bash
# A/B pass for level 0: its parity tests (schedules l0g16 / l0g7c3 / the
# adaptive default, the level-0 test, full-size configs 2 and 5), then the
# iso-profile script (bench, short bench, exclusive kernel times).
TAG=${1:-l0}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/iso/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -k "l0 or level0 or rlc16 or config2 or config5" > $O/tests.log 2>&1 || { grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_iso_prof.sh $TAG "$@"
