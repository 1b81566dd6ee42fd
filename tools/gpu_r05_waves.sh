#!/bin/bash
# Round-5 call: the level-0 Miller kernel's time against its wave count
# (one launch replayed alone, isolated_kernel_ms), for launches of 1..16
# caller batches -- how fast a wave runs alone on its SIMD vs two per SIMD.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r5waves
mkdir -p $O
for M in 1 2 4 6 8 12 16; do
  f=$O/m$M.json
  timeout -k 10 300 python3 -u bench.py --no-cpu --api-batches 0 --latency 0 --inflight 1 --merge $M --steps $M --warmup 0 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));k=d['isolated_kernel_ms'];print('m$M', d['config'].get('rlc_chunk'), k.get('k_miller_hex<MILLER_L0>'), round(d['value']))"
done
