#!/bin/bash
# Round-5 call: the GPU suite at the current build, then the driver's bench
# command (latency side key with and without the express slot).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_tests.sh r5t3 || exit 1
mkdir -p gpurun_out/r5drv2
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5drv2/driver.json 2> gpurun_out/r5drv2/driver.err || { tail -20 gpurun_out/r5drv2/driver.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5drv2/driver.json'));k=d['isolated_kernel_ms'];print('driver', d['value'], d['roofline']['frac'], d['api_pipeline']['value'], {x: k[x] for x in k if 'sgb' in x or 'clear' in x or 'miller' in x});print(json.dumps(d['small_batch_latency']))"
