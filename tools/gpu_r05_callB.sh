#!/bin/bash
# Round-5 call: parity gate of the product, A/B of the batched-subgroup
# variants and the (-x, y) operand change against HEAD's build, the driver's
# bench command (latency side key included) and config 4 via tbg_multi.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r5drv
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_config2_full_batch_matches_oracle" \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5drv/gate_product.log 2>&1 || { tail -30 gpurun_out/r5drv/gate_product.log; exit 1; }
tail -1 gpurun_out/r5drv/gate_product.log
bash tools/gpu_r05_ab.sh r5sgb product varlib/head.so varlib/s2.so varlib/m1024.so || exit 1
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5drv/driver.json 2> gpurun_out/r5drv/driver.err || { tail -20 gpurun_out/r5drv/driver.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5drv/driver.json'));print('driver', d['value'], d['roofline']['frac'], d['roofline']['frac_clock_derived'], d['api_pipeline']['value'], d['cpu_baseline']['value'], json.dumps(d['small_batch_latency']))"
timeout -k 10 600 python3 -u bench.py --workload config4 --multi-contexts 8 --steps 3 --inject 0.01 > gpurun_out/r5drv/config4_multi.json 2> gpurun_out/r5drv/config4_multi.err || { tail -20 gpurun_out/r5drv/config4_multi.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r5drv/config4_multi.json'));print('c4multi', d['value'], d['exact'], json.dumps(d['host_side']))"
