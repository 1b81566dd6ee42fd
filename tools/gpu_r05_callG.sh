#!/bin/bash
# Round-5 call: shape / headline / parity GPU tests at the fitted level-0
# shape model, then a kernel trace + timeline of the driver's 20-step
# command and of the 48-step one (the 20-step gap), and config 3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t7 "tests/test_gpu_shape.py tests/test_gpu_headline.py tests/test_gpu_parity.py" || exit 1
bash tools/gpu_r05_trace.sh r5tr20 || exit 1
mkdir -p gpurun_out/r5c3
timeout -k 10 300 python3 -u bench.py --workload config3 --steps 6 --warmup 2 --no-cpu --api-batches 0 --latency 0 > gpurun_out/r5c3/c3.json 2> gpurun_out/r5c3/c3.err || { tail -5 gpurun_out/r5c3/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5c3/c3.json'));k=d['isolated_kernel_ms'];print('c3', d['value'], d['config'].get('rlc_chunk'), k.get('k_miller_hex<MILLER_L0>'))"
